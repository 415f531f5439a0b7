set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "start $(date)"; rocm-smi --showproductname 2>&1 | head -5 || true
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" > gpurun_out/t1.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench1.err; cat gpurun_out/bench1.json
