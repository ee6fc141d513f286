#!/usr/bin/env python3
"""Lab build of the product gemm.hip with preprocessor overrides (tool only):
compile csrc/gemm.hip with -D flags and link it with the other objects into
tools/gemm_lab/libnewsrec_<name>.so for tools/gemm_ab.py.

    python tools/gemm_lab/build_define.py ho16 NR_GEMM_HANDOFF=16
"""
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
CSRC = REPO / "news_recommendation_project_v2_amd" / "csrc"
OUT = Path(__file__).resolve().parent


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    build = OUT / "build"
    build.mkdir(exist_ok=True)
    obj = build / f"gemm_{name}.o"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I", str(CSRC),
                    *[f"-D{d}" for d in defs], "-c", str(CSRC / "gemm.hip"), "-o", str(obj)], check=True)
    objs = [str(p) for p in sorted((CSRC / "build").glob("*.o")) if p.name != "gemm.o"]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", str(obj), *objs, "-ldl",
                    "-o", str(OUT / f"libnewsrec_{name}.so")], check=True)
    print("built", name, defs)


if __name__ == "__main__":
    sys.exit(main())
