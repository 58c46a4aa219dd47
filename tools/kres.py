"""Per-kernel register / LDS / spill summary of one HIP source (hipcc -Rpass-analysis).
    python tools/kres.py onepose_amd/csrc/gemm.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-w",
                    "-fPIC", "-c", src, "-o", "/tmp/_kres.o",
                    "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur = None
rows = []
for line in r.stderr.splitlines():
    m = re.search(r"remark: (?:.*?)\s(Name|VGPRs|AGPRs|Occupancy \[waves/SIMD\]|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
dem = subprocess.run(["c++filt"], input="\n".join(x["name"] for x in rows),
                     capture_output=True, text=True).stdout.splitlines()
for x, d in zip(rows, dem):
    d = d.replace("onepose::(anonymous namespace)::", "")
    if flt not in d:
        continue
    print(f"{x.get('VGPRs','?'):>4}v {x.get('AGPRs','?'):>3}a occ {x.get('Occupancy [waves/SIMD]','?')} "
          f"spill {x.get('VGPRs Spill','?')}/{x.get('SGPRs Spill','?')} lds {x.get('LDS Size [bytes/block]','?'):>6}  {d[:150]}")
