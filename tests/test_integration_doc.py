"""The C example in INTEGRATION.md compiles against include/raptor_amd.h (it did
not: `rc` was never declared).  MPI is not in the image: a three-line stand-in declares the two
MPI names the example uses; everything else is the header as shipped."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MPI_STANDIN = """typedef int MPI_Comm;
#define MPI_COMM_WORLD 0
#define MPI_BYTE 1
static int MPI_Bcast(void* b, int n, int t, int root, MPI_Comm c) { (void)b; (void)n; (void)t; (void)root; (void)c; return 0; }
"""


def test_integration_c_example_compiles(tmp_path):
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```c\n(.*?)```", doc, re.S)
    assert blocks, "no C example in INTEGRATION.md"
    src = tmp_path / "example.c"
    body = blocks[0].replace('#include "raptor_amd.h"', '#include "raptor_amd.h"\n' + MPI_STANDIN)
    src.write_text(body)
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-Wno-unused-function", "-fsyntax-only",
                        "-I", os.path.join(ROOT, "include"), str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_cxx_header_compiles_standalone(tmp_path):
    src = tmp_path / "facade.cpp"
    src.write_text('#include "raptor_amd.hpp"\nint main() { return raptor_amd::ParMultilevel::options == nullptr; }\n')
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                        "-I", os.path.join(ROOT, "include"), str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
