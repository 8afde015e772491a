#!/usr/bin/env python3
"""gfx950 ISA checks of the LDS-DMA pipelines (no GPU): in every
k_gemm3 / k_gemm2_f32 instantiation, no `s_waitcnt vmcnt(0)` may sit between
the global_load_lds of the next K step and the first ds_read of the current
one (hipcc drains the DMA pipeline there when the reads' type may alias the
DMA's, e.g. HIP's float4 struct; cdna_hip_programming.md §5 trap 4).
Usage: tools/isa_lint.py [FILE.hip] -> prints offenders, exit 1 if any."""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def gemm_drains(asm: str, pattern: str = "k_gemm"):
    out = {}
    for m in re.finditer(r"^(_Z\S*):\s*;", asm, re.M):
        nm = m.group(1)
        if pattern not in nm:
            continue
        end = asm.index(".Lfunc_end", m.end())
        lines = [l.strip() for l in asm[m.end():end].split("\n")]
        bad, last = 0, -10**9
        for i, l in enumerate(lines):
            if l.startswith("global_load_lds"):
                last = i
            elif l.startswith("s_waitcnt") and "vmcnt(0)" in l and i - last < 40:
                nxt = next((x for x in lines[i + 1:i + 8] if x.startswith(("ds_read", "s_barrier"))), "")
                bad += nxt.startswith("ds_read")
        out[nm] = bad
    return out


def main():
    src = Path(sys.argv[1]) if len(sys.argv) > 1 else REPO / "fhe-icp_amd" / "csrc" / "bert.hip"
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--save-temps", "-c", "-o",
                        f"{d}/x.o", str(src)], cwd=d, check=True, capture_output=True)
        asm = next(Path(d).glob("*gfx950.s")).read_text()
    res = gemm_drains(asm)
    for nm, bad in res.items():
        print(f"{bad} {nm}")
    sys.exit(1 if not res or any(res.values()) else 0)


if __name__ == "__main__":
    main()
