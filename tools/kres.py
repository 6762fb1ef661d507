"""Per-kernel resource usage of a HIP source (hipcc -Rpass-analysis=kernel-resource-usage),
one line per kernel: VGPRs, AGPRs, scratch bytes, occupancy (waves/SIMD), LDS.
usage: python tools/kres.py SOURCE.hip [substring-filter]"""
import re
import subprocess
import sys

import os
src = os.path.abspath(sys.argv[1])
filt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I/root/repo/include",
                    "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                   capture_output=True, text=True, cwd="/tmp")
cur = None
rows = {}
for line in r.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for name, d in rows.items():
    dm = subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
    dm = re.sub(r"\(.*", "", dm)
    if filt in dm:
        print(f"{d.get('VGPRs','?'):>4} v {d.get('AGPRs','?'):>3} a {d.get('ScratchSize [bytes/lane]','?'):>4} scr "
              f"occ {d.get('Occupancy [waves/SIMD]','?'):>2} lds {d.get('LDS Size [bytes/block]','?'):>6}  {dm}")
