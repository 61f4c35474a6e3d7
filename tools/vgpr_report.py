"""Register report of one library source's kernels (hipcc -Rpass-analysis=kernel-resource-usage), one line per kernel:
VGPRs, AGPRs, spills, occupancy, LDS.  Usage: python tools/vgpr_report.py k_direct.hip -DPGPU_MODE=0 [-DX=1 ...]"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "pinot_amd", "csrc")


def main():
    src, defs = sys.argv[1], sys.argv[2:]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
           "-Rpass-analysis=kernel-resource-usage", "-c", os.path.join(CSRC, src), "-o", "/tmp/vgpr_report.o"] + defs
    out = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True).stdout
    cur = None
    rows = []
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            if "error" in line:
                print(line)
            continue
        txt = m.group(1).strip()
        if txt.startswith("Function Name:"):
            cur = {"name": txt.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        name = subprocess.run(["c++filt", r["name"]], stdout=subprocess.PIPE, text=True).stdout.strip()
        name = name.replace("pgpu::", "").replace("(pgpu::KParams)", "")
        print("%-70s vgpr %3s agpr %3s vspill %3s sspill %3s occ %s lds %s" % (
            name[:70], r.get("VGPRs"), r.get("AGPRs"), r.get("VGPRs Spill"), r.get("SGPRs Spill"),
            r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]")))


if __name__ == "__main__":
    main()
