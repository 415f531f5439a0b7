"""Kernel resources from a device assembly file (hipcc --cuda-device-only -S): name, VGPRs,
SGPRs, scratch bytes, LDS.  Usage: kres.py file.s [substring ...]"""
import re
import sys


def main(path, subs):
    cur, out = None, []
    for line in open(path):
        m = re.match(r"\s*\.amdhsa_kernel (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            continue
        if cur is None:
            continue
        for key, tag in (("vgpr", "next_free_vgpr"), ("sgpr", "next_free_sgpr"),
                         ("scratch", "private_segment_fixed_size"), ("lds", "group_segment_fixed_size")):
            m = re.match(rf"\s*\.amdhsa_{tag} (\d+)", line)
            if m:
                cur[key] = int(m.group(1))
        if ".end_amdhsa_kernel" in line:
            out.append(cur)
            cur = None
    for k in out:
        nm = k["name"].replace("_ZN3amg12_GLOBAL__N_1", "")
        if subs and not any(s in nm for s in subs):
            continue
        print(f"{nm[:70]:70s} vgpr {k.get('vgpr', -1):3d} sgpr {k.get('sgpr', -1):3d} "
              f"scratch {k.get('scratch', -1):3d} lds {k.get('lds', -1)}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
