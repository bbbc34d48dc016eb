"""Kernel resource usage (SGPRs, VGPRs, spills, occupancy, LDS) of one HIP source, from
hipcc -Rpass-analysis=kernel-resource-usage.

  python tools/kres.py tsbb15-3d-reconstruction-project_amd/csrc/np_sampler.hip [name-filter]
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    extra = sys.argv[3:]
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
           "-fno-slp-vectorize", "-I" + os.path.join(REPO, "include"), "-c", os.path.abspath(src), "-o",
           "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"] + extra
    p = subprocess.run(cmd, capture_output=True, text=True, cwd=os.path.dirname(os.path.abspath(src)))
    cur = None
    rows = {}
    for line in p.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\S+) \[", line)
        if m and cur:
            rows[cur][m.group(1).strip()] = m.group(2)
    if p.returncode:
        print(p.stderr[-3000:])
    for k, v in rows.items():
        if filt in k:
            print(f"{k[:70]:70s} sgpr {v.get('TotalSGPRs')} (spill {v.get('SGPRs Spill')}) "
                  f"vgpr {v.get('VGPRs')} (spill {v.get('VGPRs Spill')}) occ {v.get('Occupancy [waves/SIMD]')} "
                  f"lds {v.get('LDS Size [bytes/block]')} scratch {v.get('ScratchSize [bytes/lane]')}")


if __name__ == "__main__":
    main()
