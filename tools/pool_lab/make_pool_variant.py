#!/usr/bin/env python3
"""Lab variants of pool_score_kernel (tool only, never shipped): patch a COPY of
csrc/pool_score.hip with one named change, link it with the other objects into
tools/pool_lab/libnewsrec_<name>.so for tools/pool_ab.py.

    python tools/pool_lab/make_pool_variant.py wg64 lat16 lds6
"""
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
CSRC = REPO / "news_recommendation_project_v2_amd" / "csrc"
OUT = Path(__file__).resolve().parent

LAUNCH = "hipLaunchKernelGGL((pool_score_kernel<T, POOL, 1024>), dim3((unsigned)blocks), dim3(256), 0, s,"


def lds_cap(kb):
    # dynamic LDS (unused) so that at most 160 / kb workgroups fit on a CU
    return [(LAUNCH, LAUNCH.replace("dim3(256), 0, s", f"dim3(256), {kb * 1024}, s"))]


VARIANTS = {
    "base": [],
    # one impression per 64-thread workgroup: no waiting on a workgroup's slowest wave
    "wg64": [("const int64_t imp = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);",
              "const int64_t imp = (int64_t)blockIdx.x;"),
             ("const int64_t blocks = (n_imp + 3) / 4;", "const int64_t blocks = n_imp;"),
             (LAUNCH, LAUNCH.replace("dim3(256), 0, s", "dim3(64), 0, s")),
             ("__launch_bounds__(256) void pool_score_kernel", "__launch_bounds__(64) void pool_score_kernel")],
    # 16 history rows in flight per wave (bf16 latent)
    "lat16": [("template <> struct PoolCfg<__bf16, NR_POOL_LATENT> { static constexpr int R = 8; };",
               "template <> struct PoolCfg<__bf16, NR_POOL_LATENT> { static constexpr int R = 16; };")],
    "lat4": [("template <> struct PoolCfg<__bf16, NR_POOL_LATENT> { static constexpr int R = 8; };",
              "template <> struct PoolCfg<__bf16, NR_POOL_LATENT> { static constexpr int R = 4; };")],
    # the first 64 candidate ids and inverse norms loaded before the history loop
    "cpre": [("  // ---------------- history pooling ----------------\n  const int64_t h0 = hoff[imp], h1 = hoff[imp + 1];",
              "  const int64_t c0p = coff ? coff[imp] : 0, c1p = coff ? coff[imp + 1] : 0;\n"
              "  const int cnt0 = (int)min((int64_t)64, c1p - c0p);\n"
              "  const int pidx = lane < cnt0 ? cidx[c0p + lane] : 0;\n"
              "  const float pinv = lane < cnt0 ? cinv[pidx] : 0.f;\n"
              "  // ---------------- history pooling ----------------\n  const int64_t h0 = hoff[imp], h1 = hoff[imp + 1];"),
             ("    const int myidx = lane < cnt ? cidx[base + lane] : 0;\n    const float myinv = lane < cnt ? cinv[myidx] : 0.f;",
              "    const int myidx = base == c0 ? pidx : (lane < cnt ? cidx[base + lane] : 0);\n"
              "    const float myinv = base == c0 ? pinv : (lane < cnt ? cinv[myidx] : 0.f);")],
    "lat32": [("template <> struct PoolCfg<__bf16, NR_POOL_LATENT> { static constexpr int R = 8; };",
               "template <> struct PoolCfg<__bf16, NR_POOL_LATENT> { static constexpr int R = 32; };")],
    "fin8": [("template <> struct PoolCfg<__bf16, NR_POOL_FINAL> { static constexpr int R = 4; };",
              "template <> struct PoolCfg<__bf16, NR_POOL_FINAL> { static constexpr int R = 8; };")],
    # 8 candidate rows in flight per wave (two transpose-reduces)
    "g8": [("  constexpr int G = 4;", "  constexpr int G = 8;"),
           ("""      const float b = reduce4(d, lane);
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const float t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b), 16 * q));""",
            """      float b[G / 4];
#pragma unroll
      for (int h = 0; h < G / 4; ++h) {
        const float dd[4] = {d[4 * h], d[4 * h + 1], d[4 * h + 2], d[4 * h + 3]};
        b[h] = reduce4(dd, lane);
      }
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const float t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b[q / 4]), 16 * (q % 4)));""")],
    # non-temporal (streaming) loads for the gathered table rows
    "nt": [("  for (int j = 0; j < RowFmt<T, DIM>::NL; ++j) r[j] = p[j * 64];",
            "  for (int j = 0; j < RowFmt<T, DIM>::NL; ++j) {\n"
            "    auto t = __builtin_nontemporal_load(reinterpret_cast<const __attribute__((ext_vector_type(4))) unsigned int*>(p + j * 64));\n"
            "    r[j] = make_uint4(t.x, t.y, t.z, t.w);\n  }")],
    "lds4": lds_cap(40),
    "lds5": lds_cap(32),
    "lds6": lds_cap(26),
    "lds8": lds_cap(20),
}


def build(name):
    """name: one variant or several joined by '+' (patches applied in order)."""
    src = (CSRC / "pool_score.hip").read_text()
    for old, new in [pt for part in name.split("+") for pt in VARIANTS[part]]:
        if old not in src:
            raise SystemExit(f"{name}: patch anchor not found: {old[:60]!r}")
        src = src.replace(old, new)
    d = OUT / "build"
    d.mkdir(exist_ok=True)
    cpy = d / f"pool_score_{name}.hip"
    cpy.write_text(src)
    obj = d / f"pool_score_{name}.o"
    hip = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{CSRC}"]
    subprocess.run(hip + ["-c", str(cpy), "-o", str(obj)], check=True)
    others = [p for p in (CSRC / "build").glob("*.o") if p.name != "pool_score.o"]
    lib = OUT / f"libnewsrec_{name}.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", str(obj), *map(str, others),
                    "-o", str(lib)], check=True)
    print(lib)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(VARIANTS):
        build(n)
