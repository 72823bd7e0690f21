"""Register / LDS / occupancy table of every kernel in one .hip file (hipcc resource remarks).

  python tools/kres.py csrc/kernels/lstm_persistent.hip [name-substring]
"""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=fast",
           "-munsafe-fp-atomics", f"-I{ROOT}/csrc/kernels", "-c", src, "-o", "/tmp/kres.o",
           "-Rpass-analysis=kernel-resource-usage"] + os.environ.get("KRES_FLAGS", "").split()
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)",
                      line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None:
            cur[k.split(" [")[0]] = v
    for r in rows:
        if pat in r["name"]:
            print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>3} a  spill {r.get('VGPRs Spill', '?'):>3}  "
                  f"occ {r.get('Occupancy', '?')}  lds {r.get('LDS Size', '?'):>6}  {r['name'][:110]}")


if __name__ == "__main__":
    main()
