"""Per-kernel register / occupancy report of one HIP translation unit (gfx950), from the
compiler's resource-usage remarks -- used to check that an epilogue or prologue change did not
cost a kernel instantiation its occupancy:

    python scripts/kernel_resources.py csrc/kernels/conv_fwd.hip [filter]
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def resources(src: str, include: str = str(ROOT / "csrc" / "include")) -> dict:
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", include, "-c", src,
           "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    out, cur = {}, None
    for line in res.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"(VGPRs|AGPRs|Occupancy \[waves/SIMD\]|VGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            out[cur][m.group(1).split(" ")[0] + ("_spill" if "Spill" in m.group(1) else "")] = int(m.group(2))
    return out


def main():
    src = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    inc = sys.argv[3] if len(sys.argv) > 3 else str(ROOT / "csrc" / "include")
    for k, v in sorted(resources(src, inc).items()):
        if flt in k:
            print(f"{k:110s} vgpr={v.get('VGPRs')} agpr={v.get('AGPRs')} occ={v.get('Occupancy')} "
                  f"spill={v.get('VGPRs_spill')}")


if __name__ == "__main__":
    main()
