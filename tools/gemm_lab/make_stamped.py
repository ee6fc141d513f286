#!/usr/bin/env python3
"""Diagnostic build (tool only, never shipped): patch a COPY of csrc/gemm.hip so
the persistent bf16 kernel (gemm256t_kernel) accumulates s_memtime phase
durations per workgroup in registers (wave 0) and writes them once at its end
into a buffer set by lab_set_stamps(); link it with the other objects into
tools/gemm_lab/libnewsrec_stamped.so.  Phases per tile:
  main  = accumulators seeded -> last K step done
  epi   = -> epilogue computed, stores issued
  top   = -> next tile's accumulators seeded
The stamps read the shader clock only (no memory traffic inside the loop)."""
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
CSRC = REPO / "news_recommendation_project_v2_amd" / "csrc"
OUT = Path(__file__).resolve().parent


def patch(src: str) -> str:
    """Clock stamps only (round 6): s_memtime / s_memrealtime once at the top of the
    persistent loop and once at the kernel's end, per workgroup, plus its unit count.
    (Round 2's per-phase stamps anchored on a K loop that has since been restructured.)"""
    def sub(old, new):
        nonlocal src
        assert src.count(old) == 1, old
        src = src.replace(old, new)
    sub('#include "nr_common.h"', '#include "nr_common.h"\n__device__ unsigned long long* g_lab_stamps = nullptr;')
    sub("  if (wmu == 1) __builtin_amdgcn_s_barrier();  // skew the wave groups by one barrier\n  while (true) {\n",
        "  if (wmu == 1) __builtin_amdgcn_s_barrier();  // skew the wave groups by one barrier\n"
        "  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime(), ck0 = __builtin_amdgcn_s_memtime();\n"
        "  unsigned long long s_n = 0;\n"
        "  while (true) {\n    ++s_n;\n")
    sub("    kloop(std::true_type{}, false, 0u, 0u);\n  }\n#undef NR_PHASE_SYNC_MMA\n}",
        "    kloop(std::true_type{}, false, 0u, 0u);\n  }\n"
        "  const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime(), ck1 = __builtin_amdgcn_s_memtime();\n"
        "  if (tid == 0 && g_lab_stamps) {\n"
        "    unsigned long long* o = g_lab_stamps + blockIdx.x * 8;\n"
        "    o[0] = 0; o[1] = 0; o[2] = 0; o[3] = 0; o[4] = s_n; o[5] = ck1 - ck0; o[6] = rt1 - rt0;\n"
        "  }\n#undef NR_PHASE_SYNC_MMA\n}")
    src += '\nextern "C" int lab_set_stamps(void* p) {\n  return hipMemcpyToSymbol(HIP_SYMBOL(g_lab_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1;\n}\n'
    return src


def main():
    build = OUT / "build"
    build.mkdir(exist_ok=True)
    (build / "gemm_stamped.hip").write_text(patch((CSRC / "gemm.hip").read_text()))
    inc = ["-I", str(CSRC)]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *inc, "-c",
                    str(build / "gemm_stamped.hip"), "-o", str(build / "gemm_stamped.o")], check=True)
    objs = [str(p) for p in sorted((CSRC / "build").glob("*.o")) if p.name != "gemm.o"]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", str(build / "gemm_stamped.o"),
                    *objs, "-o", str(OUT / "libnewsrec_stamped.so")], check=True)
    print("built")


if __name__ == "__main__":
    sys.exit(main())
