#!/usr/bin/env python3
"""Lab variants of the persistent GEMM (tool only, never shipped): patch a COPY
of csrc/gemm.hip with one named change, link it with the other objects into
tools/gemm_lab/libnewsrec_<name>.so for tools/gemm_ab.py.

    python tools/gemm_lab/make_variant.py flatdma

Each variant is a set of exact-text patches against gemm.hip AS IT WAS when
that A/B ran (recorded in DESIGN.md §3.2 / profiles/round*/): adopted ones
(quarters, dma2, fastexp) are in the source now, and patches written against
an older main loop no longer apply (the script then stops at the failing
assert instead of building a wrong library).

The lab-only kernels (the MF32 32x32x16 branches of gemm256t_kernel and the
4-wave gemm256w4_kernel, DESIGN.md §3.2b: measured, not adopted) are not in the
product source: variants listed in OVERLAY first apply
patches/lab_kernels.patch (a unified diff against csrc/gemm.hip) to the copy.
"""
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
CSRC = REPO / "news_recommendation_project_v2_amd" / "csrc"
OUT = Path(__file__).resolve().parent

VARIANTS = {
    # operand DMA units cut into the quarters each phase finishes reading (A: one
    # 64-row qm quarter of both wave-group halves, B: one 32-row qn quarter of
    # all four wn slices), issued P2: A0+B0, P3: B1, P4: A1 (was P3: B0, P4: B1+A0+A1)
    "quarters": [
        ("  const int rl = 16 * wave + (lane >> 3);\n",
         "  const int rl = 16 * wave + (lane >> 3);\n"
         "  const int qa = (wave >> 2) * 128 + (wave & 3) * 16, qb = (wave >> 1) * 64 + (wave & 1) * 16;\n"),
        ("oA[h][j] = min(mb + (uint32_t)(128 * h + 8 * j + rl), mlast) * ldab + chunk(j);",
         "oA[h][j] = min(mb + (uint32_t)(qa + 64 * h + 8 * j + (lane >> 3)), mlast) * ldab + chunk(j);"),
        ("oB[h][j] = (nb + (uint32_t)(128 * h + 8 * j + rl)) * ldwb + chunk(j);",
         "oB[h][j] = (nb + (uint32_t)(qb + 32 * h + 8 * j + (lane >> 3))) * ldwb + chunk(j);"),
        ("    unsigned char* sa = smem + stage * G2_STAGE + (128 * h + 16 * wave) * 128;\n#pragma unroll\n    for (int j = 0; j < 2; ++j)\n      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA,",
         "    unsigned char* sa = smem + stage * G2_STAGE + (qa + 64 * h) * 128;\n#pragma unroll\n    for (int j = 0; j < 2; ++j)\n      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA,"),
        ("    unsigned char* sb = smem + stage * G2_STAGE + G2BM * 128 + (128 * h + 16 * wave) * 128;\n#pragma unroll\n    for (int j = 0; j < 2; ++j)\n      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW,",
         "    unsigned char* sb = smem + stage * G2_STAGE + G2BM * 128 + (qb + 32 * h) * 128;\n#pragma unroll\n    for (int j = 0; j < 2; ++j)\n      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW,"),
        ("""    readB(st, 1, fb1);
    NR_PHASE_SYNC_MMA(0, 1, fb1)
    readA(st, 1);
    if (pf) {
      if (kt + 2 == nk) {
        set_offA(nm0);
        set_offB(nn0);
        dma_bias(nn0);
      }
      dmaB(0, st, kf);
    }
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    if (pf) {
      dmaB(1, st, kf);
      dmaA(0, st, kf);
      dmaA(1, st, kf);""",
         """    readB(st, 1, fb1);
    if (pf) {
      if (kt + 2 == nk) {
        set_offA(nm0);
        set_offB(nn0);
        dma_bias(nn0);
      }
      dmaA(0, st, kf);
      dmaB(0, st, kf);
    }
    NR_PHASE_SYNC_MMA(0, 1, fb1)
    readA(st, 1);
    if (pf) dmaB(1, st, kf);
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    if (pf) {
      dmaA(1, st, kf);"""),
    ],
    # operand DMAs as global_load_lds (FLAT encoding) instead of buffer loads
    "flatdma": [
        ("__builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(sa + 8 * j * 128), 16, oA[h][j], kt * (BK * 2), 0, 0);",
         "__builtin_amdgcn_global_load_lds((g_void*)((const char*)A + oA[h][j] + kt * (BK * 2)), "
         "(lds_void*)(sa + 8 * j * 128), 16, 0, 0);"),
        ("__builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(sb + 8 * j * 128), 16, oB[h][j], kt * (BK * 2), 0, 0);",
         "__builtin_amdgcn_global_load_lds((g_void*)((const char*)W + oB[h][j] + kt * (BK * 2)), "
         "(lds_void*)(sb + 8 * j * 128), 16, 0, 0);"),
    ],
    # the P4 operand waits as opaque inline asm (the compiler no longer sees them)
    "asmwait": [
        ("    if (pb) __builtin_amdgcn_s_waitcnt(kVmcnt2);\n    else __builtin_amdgcn_s_waitcnt(kVmcnt0);",
         '    if (pb) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");\n'
         '    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");'),
    ],
    # operand refills spread 2 pieces per phase: P1 A1 (deferred from the previous step,
    # into the other stage), P2 A0, P3 B0, P4 B1 (shipped: P2 A0+B0, P3 B1, P4 A1);
    # P4 then leaves 6 pieces in flight (vmcnt(6), 9 with the LN slices)
    "dma2": [
        ("constexpr unsigned kVmcnt0 = 0x0F70, kVmcnt8 = 0x0F78, kVmcnt11 = 0x0F7B;",
         "constexpr unsigned kVmcnt0 = 0x0F70, kVmcnt8 = 0x0F78, kVmcnt11 = 0x0F7B, kVmcnt6 = 0x0F76, kVmcnt9 = 0x0F79;"),
        ("""  auto kstep = [&](int kt, int st, bool more, uint32_t nm0, uint32_t nn0) {
    const bool pf = kt + 2 < nk || more;
    const int kf = kt + 2 < nk ? kt + 2 : kt + 2 - nk;
    readA(st, 0);
    readB(st, 0, fb0);
    NR_PHASE_SYNC_MMA(0, 0, fb0)
    readB(st, 1, fb1);
    if (pf) {
      if (kt + 2 == nk) {
        set_offA(nm0);
        set_offB(nn0);
        dma_bias(nn0);
      }
      dmaA(0, st, kf);
      dmaB(0, st, kf);
    }
    NR_PHASE_SYNC_MMA(0, 1, fb1)
    readA(st, 1);
    if (pf) dmaB(1, st, kf);
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    if (pf) {
      dmaA(1, st, kf);
      if (LNF && kt + 2 == nk) {
        // the next tile's LN slices after its step-0 DMAs: they get a whole K step
        dma_ln(lslot ^ 1, nm0, nn0);
        __builtin_amdgcn_s_waitcnt(kVmcnt11);
      } else {
        __builtin_amdgcn_s_waitcnt(kVmcnt8);  // step kt + 1 landed; kt + 2 (8 DMAs) may fly
      }
    } else {
      __builtin_amdgcn_s_waitcnt(kVmcnt0);
    }""",
         """  bool a1p = false;  // the previous step's A1 refill (stage st ^ 1, step a1k), issued in this step's P1
  int a1k = 0;
  auto kstep = [&](int kt, int st, bool more, uint32_t nm0, uint32_t nn0) {
    const bool pf = kt + 2 < nk || more;
    const int kf = kt + 2 < nk ? kt + 2 : kt + 2 - nk;
    readA(st, 0);
    readB(st, 0, fb0);
    if (a1p) dmaA(1, st ^ 1, a1k);
    NR_PHASE_SYNC_MMA(0, 0, fb0)
    readB(st, 1, fb1);
    if (pf) {
      if (kt + 2 == nk) {
        set_offA(nm0);
        set_offB(nn0);
        dma_bias(nn0);
      }
      dmaA(0, st, kf);
    }
    NR_PHASE_SYNC_MMA(0, 1, fb1)
    readA(st, 1);
    if (pf) dmaB(0, st, kf);
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    if (pf) {
      dmaB(1, st, kf);
      if (LNF && kt + 2 == nk) {
        dma_ln(lslot ^ 1, nm0, nn0);
        __builtin_amdgcn_s_waitcnt(kVmcnt9);
      } else {
        __builtin_amdgcn_s_waitcnt(kVmcnt6);  // step kt + 1 landed (incl. its A1 from P1); 6 of kt + 2 fly
      }
    } else {
      __builtin_amdgcn_s_waitcnt(kVmcnt0);
    }
    a1p = pf;
    a1k = kf;"""),
    ],
    # the persistent kernel's EXP / SOFTMAX64 epilogues on v_exp_f32 (x log2 e), not the
    # accurate expf (stamps: the S epilogue 13.5 k cycles per tile vs 4.2 k plain)
    "fastexp": [
        ("__device__ __forceinline__ float epi_exp(float x) { return expf(x); }",
         "__device__ __forceinline__ float epi_exp(float x) { return __expf(x); }"),
    ],
    # next step's B0 fragments read in P4 (into the B1 registers, free there; the two
    # B fragment sets swap roles every step, K loop unrolled by 2), landed by a counted
    # vmcnt in P3: LDS reads per phase 8 / 4 / 8 / 4 instead of 12 / 4 / 8 / 0
    "rb": [
        ("constexpr unsigned kVmcnt0 = 0x0F70, kVmcnt8 = 0x0F78, kVmcnt11 = 0x0F7B;",
         "constexpr unsigned kVmcnt0 = 0x0F70, kVmcnt8 = 0x0F78, kVmcnt11 = 0x0F7B, kVmcnt10 = 0x0F7A;"),
        ("""  auto kstep = [&](int kt, int st, bool more, uint32_t nm0, uint32_t nn0) {
    const bool pf = kt + 2 < nk || more;
    const int kf = kt + 2 < nk ? kt + 2 : kt + 2 - nk;
    readA(st, 0);
    readB(st, 0, fb0);
    NR_PHASE_SYNC_MMA(0, 0, fb0)
    readB(st, 1, fb1);""",
         """  auto kstep = [&](int kt, int st, bool more, uint32_t nm0, uint32_t nn0, frag_t (&fx)[2][2], frag_t (&fy)[2][2]) {
    const bool pf = kt + 2 < nk || more;
    const bool nx = kt + 1 < nk || more;
    const int kf = kt + 2 < nk ? kt + 2 : kt + 2 - nk;
    readA(st, 0);
    NR_PHASE_SYNC_MMA(0, 0, fx)
    readB(st, 1, fy);"""),
        ("""    NR_PHASE_SYNC_MMA(0, 1, fb1)
    readA(st, 1);
    if (pf) dmaB(1, st, kf);
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    if (pf) {""",
         """    NR_PHASE_SYNC_MMA(0, 1, fy)
    readA(st, 1);
    if (pf) dmaB(1, st, kf);
    if (nx) {
      if (pf) __builtin_amdgcn_s_waitcnt(kVmcnt10);  // step kt + 1's B0 quarter landed (10+ younger pieces)
      else __builtin_amdgcn_s_waitcnt(kVmcnt0);
    }
    NR_PHASE_SYNC_MMA(1, 1, fy)
    if (nx) readB(st ^ 1, 0, fy);  // step kt + 1's B0 (read after the barrier that follows every wave's wait)
    if (pf) {"""),
        ("""    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
    mma(1, 0, fb0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };""",
         """    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
    mma(1, 0, fx);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };"""),
        ("""  if (wmu == 1) __builtin_amdgcn_s_barrier();  // skew the wave groups by one barrier
  int st = 0;
  while (true) {""",
         """  if (wmu == 1) __builtin_amdgcn_s_barrier();  // skew the wave groups by one barrier
  int st = 0;
  readB(0, 0, fb0);
  while (true) {"""),
        ("""    for (int kt = 0; kt < nk; ++kt) {
      kstep(kt, st, more, nm0, nn0);
      st ^= 1;
    }

    if (wmu == 0) __builtin_amdgcn_s_barrier();  // realign: group 1 has finished its last MFMA phase""",
         """    for (int kt = 0; kt < nk; kt += 2) {  // nk even (host)
      kstep(kt, st, more, nm0, nn0, fb0, fb1);
      kstep(kt + 1, st ^ 1, more, nm0, nn0, fb1, fb0);
    }

    if (wmu == 0) __builtin_amdgcn_s_barrier();  // realign: group 1 has finished its last MFMA phase"""),
        ("  return K >= 128 && M * lda * 2 <= kMax && N * ldw * 2 <= kMax;",
         "  return K >= 128 && K % 128 == 0 && M * lda * 2 <= kMax && N * ldw * 2 <= kMax;"),
    ],
    # rb with the next tile's step-0 B0 read at its tile top (no fragments live through the epilogue)
    "rb2": [
        ("constexpr unsigned kVmcnt0 = 0x0F70, kVmcnt8 = 0x0F78, kVmcnt11 = 0x0F7B;",
         "constexpr unsigned kVmcnt0 = 0x0F70, kVmcnt8 = 0x0F78, kVmcnt11 = 0x0F7B, kVmcnt10 = 0x0F7A;"),
        ("""  auto kstep = [&](int kt, int st, bool more, uint32_t nm0, uint32_t nn0) {
    const bool pf = kt + 2 < nk || more;
    const int kf = kt + 2 < nk ? kt + 2 : kt + 2 - nk;
    readA(st, 0);
    readB(st, 0, fb0);
    NR_PHASE_SYNC_MMA(0, 0, fb0)
    readB(st, 1, fb1);""",
         """  auto kstep = [&](int kt, int st, bool more, uint32_t nm0, uint32_t nn0, frag_t (&fx)[2][2], frag_t (&fy)[2][2]) {
    const bool pf = kt + 2 < nk || more;
    const bool nx = kt + 1 < nk || more;
    const int kf = kt + 2 < nk ? kt + 2 : kt + 2 - nk;
    readA(st, 0);
    NR_PHASE_SYNC_MMA(0, 0, fx)
    readB(st, 1, fy);"""),
        ("""    NR_PHASE_SYNC_MMA(0, 1, fb1)
    readA(st, 1);
    if (pf) dmaB(1, st, kf);
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    if (pf) {""",
         """    NR_PHASE_SYNC_MMA(0, 1, fy)
    readA(st, 1);
    if (pf) dmaB(1, st, kf);
    if (nx) {
      if (pf) __builtin_amdgcn_s_waitcnt(kVmcnt10);  // step kt + 1's B0 quarter landed (10+ younger pieces)
      else __builtin_amdgcn_s_waitcnt(kVmcnt0);
    }
    NR_PHASE_SYNC_MMA(1, 1, fy)
    if (kt + 1 < nk) readB(st ^ 1, 0, fy);  // step kt + 1's B0 (read after the barrier that follows every wave's wait)
    if (pf) {"""),
        ("""    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
    mma(1, 0, fb0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };""",
         """    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
    mma(1, 0, fx);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };"""),
        ("""  if (wmu == 1) __builtin_amdgcn_s_barrier();  // skew the wave groups by one barrier
  int st = 0;
  while (true) {""",
         """  if (wmu == 1) __builtin_amdgcn_s_barrier();  // skew the wave groups by one barrier
  int st = 0;
  const int t_first = t;
  readB(0, 0, fb0);
  while (true) {"""),
        ("""    for (int kt = 0; kt < nk; ++kt) {
      kstep(kt, st, more, nm0, nn0);
      st ^= 1;
    }

    if (wmu == 0) __builtin_amdgcn_s_barrier();  // realign: group 1 has finished its last MFMA phase""",
         """    if (t != t_first) readB(st, 0, fb0);  // the tile's step-0 B0 (not held through the epilogue)
    for (int kt = 0; kt < nk; kt += 2) {  // nk even (host)
      kstep(kt, st, more, nm0, nn0, fb0, fb1);
      kstep(kt + 1, st ^ 1, more, nm0, nn0, fb1, fb0);
    }

    if (wmu == 0) __builtin_amdgcn_s_barrier();  // realign: group 1 has finished its last MFMA phase"""),
        ("  return K >= 128 && M * lda * 2 <= kMax && N * ldw * 2 <= kMax;",
         "  return K >= 128 && K % 128 == 0 && M * lda * 2 <= kMax && N * ldw * 2 <= kMax;"),
    ],
    # on top of the shipped spread (P1 A1', P2 A0, P3 B0, P4 B1): B0 moved to the read-free P4
    "dma4": [
        ("""    readA(st, 1);
    if (pf) dmaB(0, st, kf);
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    if (pf) {
      dmaB(1, st, kf);""",
         """    readA(st, 1);
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    if (pf) {
      dmaB(0, st, kf);
      dmaB(1, st, kf);"""),
    ],
    # dma4 + the deferred A1 in P2 instead of P1 (P1: 12 reads only; P2: 4 reads + A1' + A0; P3: 8 reads; P4: B0 + B1)
    "dma6": [
        ("""    readB(st, 0, fb0);
    if (a1p) dmaA(1, st ^ 1, a1k);
    NR_PHASE_SYNC_MMA(0, 0, fb0)
    readB(st, 1, fb1);
    if (pf) {""",
         """    readB(st, 0, fb0);
    NR_PHASE_SYNC_MMA(0, 0, fb0)
    readB(st, 1, fb1);
    if (a1p) dmaA(1, st ^ 1, a1k);
    if (pf) {"""),
        ("""    readA(st, 1);
    if (pf) dmaB(0, st, kf);
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    if (pf) {
      dmaB(1, st, kf);""",
         """    readA(st, 1);
    NR_PHASE_SYNC_MMA(1, 1, fb1)
    if (pf) {
      dmaB(0, st, kf);
      dmaB(1, st, kf);"""),
    ],
    # the persistent kernel's MFMA phases without s_setprio (gemm256t only)
    "noprio_t": [
        ("""  __builtin_amdgcn_s_setprio(1);                       \\
  mma(QM, NI, FB);                                     \\
  __builtin_amdgcn_s_setprio(0);                       \\
  __builtin_amdgcn_s_barrier();
  // K step kt of the current tile (stage st).""",
         """  mma(QM, NI, FB);                                     \\
  __builtin_amdgcn_s_barrier();
  // K step kt of the current tile (stage st)."""),
    ],
    # DIAGNOSTIC (wrong results): no operand DMAs inside the K loop
    "nodma": [
        ("  auto kstep = [&](int kt, int st, bool more, uint32_t nm0, uint32_t nn0) {\n    const int ns = st ^ 1;\n"
         "    const bool pa = kt + 1 < nk || more, pb = kt + 2 < nk || more;",
         "  auto kstep = [&](int kt, int st, bool more, uint32_t nm0, uint32_t nn0) {\n    const int ns = st ^ 1;\n"
         "    const bool pa = false, pb = false;"),
    ],
    # DIAGNOSTIC (wrong results): no fragment reads (MFMA on stale registers)
    "noread": [
        ("    readA(st, 0);\n    readB(st, 0, fb0);\n    if (pa) {", "    if (pa) {"),
        ("    readB(st, 1, fb1);\n    if (pa) dmaA(1, ns, ka);", "    if (pa) dmaA(1, ns, ka);"),
        ("    readA(st, 1);\n    if (pb) {", "    if (pb) {"),
    ],
    # tile order: M-tiles per group of the persistent schedule (tile_of), 4 shipped
    "gm1": [("constexpr int kGemmGroupM = 4;", "constexpr int kGemmGroupM = 1;")],
    "gm2": [("constexpr int kGemmGroupM = 4;", "constexpr int kGemmGroupM = 2;")],
    "gm8": [("constexpr int kGemmGroupM = 4;", "constexpr int kGemmGroupM = 8;")],
    "gm16": [("constexpr int kGemmGroupM = 4;", "constexpr int kGemmGroupM = 16;")],
    # the persistent kernel's main loop and epilogue on v_mfma_f32_32x32x16_bf16 (MF32)
    "mf32": [
        ("hipLaunchKernelGGL((gemm256t_kernel<E>), grid,", "hipLaunchKernelGGL((gemm256t_kernel<E, false, true>), grid,"),
        ("hipLaunchKernelGGL((gemm256t_kernel<NR_EPI_GEGLU, true>), grid,",
         "hipLaunchKernelGGL((gemm256t_kernel<NR_EPI_GEGLU, true, true>), grid,"),
        ("hipLaunchKernelGGL((gemm256t_kernel<NR_EPI_SOFTMAX64, true>), grid,",
         "hipLaunchKernelGGL((gemm256t_kernel<NR_EPI_SOFTMAX64, true, true>), grid,"),
    ],
    # 4 waves of 128x128 per 256x256 tile on 32x32x16 MFMAs (gemm256w4_kernel)
    "w4": [
        ("hipLaunchKernelGGL((gemm256t_kernel<E>), grid, dim3(512),", "hipLaunchKernelGGL((gemm256w4_kernel<E>), grid, dim3(256),"),
        ("hipLaunchKernelGGL((gemm256t_kernel<NR_EPI_GEGLU, true>), grid, dim3(512),",
         "hipLaunchKernelGGL((gemm256w4_kernel<NR_EPI_GEGLU, true>), grid, dim3(256),"),
        ("hipLaunchKernelGGL((gemm256t_kernel<NR_EPI_SOFTMAX64, true>), grid, dim3(512),",
         "hipLaunchKernelGGL((gemm256w4_kernel<NR_EPI_SOFTMAX64, true>), grid, dim3(256),"),
    ],
    # no s_setprio around the MFMA phases
    # GEGLU epilogue: the gelu of two accumulator values at once on float2 vectors, so the
    # erfc polynomial and the affine steps issue as v_pk_fma_f32 / v_pk_mul_f32 (SGPR
    # splat coefficients) instead of scalar v_fmaak_f32; per element the same fma
    # sequence (bit-identical), rcp / exp stay scalar
    "gelu2": [
        ("__device__ __forceinline__ float epi_exp(float x) { return __expf(x); }\n",
         """__device__ __forceinline__ float epi_exp(float x) { return __expf(x); }

typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2v fma2(f32x2v a, f32x2v b, f32x2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2v gelu_erf2(f32x2v g) {
  const f32x2v x = g * 0.70710678118654752440f;
  const f32x2v z = __builtin_elementwise_abs(x);
  f32x2v t = fma2((f32x2v)0.5f, z, (f32x2v)1.0f);
  t.x = __builtin_amdgcn_rcpf(t.x);
  t.y = __builtin_amdgcn_rcpf(t.y);
  f32x2v p = (f32x2v)0.17087277f;
  p = fma2(p, t, (f32x2v)-0.82215223f);
  p = fma2(p, t, (f32x2v)1.48851587f);
  p = fma2(p, t, (f32x2v)-1.13520398f);
  p = fma2(p, t, (f32x2v)0.27886807f);
  p = fma2(p, t, (f32x2v)-0.18628806f);
  p = fma2(p, t, (f32x2v)0.09678418f);
  p = fma2(p, t, (f32x2v)0.37409196f);
  p = fma2(p, t, (f32x2v)1.00002368f);
  const f32x2v w = fma2(t, p, fma2(-z, z, (f32x2v)-1.26551223f));
  const f32x2v ans = t * (f32x2v){__expf(w.x), __expf(w.y)};
  const f32x2v pos = g * fma2((f32x2v)-0.5f, ans, (f32x2v)1.0f);
  const f32x2v neg = (0.5f * g) * ans;
  return (f32x2v){x.x >= 0.f ? pos.x : neg.x, x.y >= 0.f ? pos.y : neg.y};
}
"""),
        ("""          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = acc[mi][ni][r] * gelu_erf(acc[mi][ni + 2][r]);
          pk[ni] = uint2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};""",
         """          const f32x2v o0 = (f32x2v){acc[mi][ni][0], acc[mi][ni][1]} *
                            gelu_erf2((f32x2v){acc[mi][ni + 2][0], acc[mi][ni + 2][1]});
          const f32x2v o1 = (f32x2v){acc[mi][ni][2], acc[mi][ni][3]} *
                            gelu_erf2((f32x2v){acc[mi][ni + 2][2], acc[mi][ni + 2][3]});
          pk[ni] = uint2{pack_bf16x2(o0.x, o0.y), pack_bf16x2(o1.x, o1.y)};"""),
    ],
    # gelu2 with the two float2 chains of a 4-column group interleaved statement by
    # statement (two independent v_pk_fma_f32 chains instead of one dependent one)
    "gelu4": [
        ("__device__ __forceinline__ float epi_exp(float x) { return __expf(x); }\n",
         """__device__ __forceinline__ float epi_exp(float x) { return __expf(x); }

typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2v fma2(f32x2v a, f32x2v b, f32x2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ void gelu_erf2x2(f32x2v& g0, f32x2v& g1) {
  const f32x2v x0 = g0 * 0.70710678118654752440f, x1 = g1 * 0.70710678118654752440f;
  const f32x2v z0 = __builtin_elementwise_abs(x0), z1 = __builtin_elementwise_abs(x1);
  f32x2v t0 = fma2((f32x2v)0.5f, z0, (f32x2v)1.0f), t1 = fma2((f32x2v)0.5f, z1, (f32x2v)1.0f);
  t0.x = __builtin_amdgcn_rcpf(t0.x);
  t1.x = __builtin_amdgcn_rcpf(t1.x);
  t0.y = __builtin_amdgcn_rcpf(t0.y);
  t1.y = __builtin_amdgcn_rcpf(t1.y);
  f32x2v p0 = (f32x2v)0.17087277f, p1 = (f32x2v)0.17087277f;
#define NR_G4(c) p0 = fma2(p0, t0, (f32x2v)(c)); p1 = fma2(p1, t1, (f32x2v)(c));
  NR_G4(-0.82215223f) NR_G4(1.48851587f) NR_G4(-1.13520398f) NR_G4(0.27886807f)
  NR_G4(-0.18628806f) NR_G4(0.09678418f) NR_G4(0.37409196f) NR_G4(1.00002368f)
#undef NR_G4
  const f32x2v w0 = fma2(t0, p0, fma2(-z0, z0, (f32x2v)-1.26551223f));
  const f32x2v w1 = fma2(t1, p1, fma2(-z1, z1, (f32x2v)-1.26551223f));
  const f32x2v a0 = t0 * (f32x2v){__expf(w0.x), __expf(w0.y)};
  const f32x2v a1 = t1 * (f32x2v){__expf(w1.x), __expf(w1.y)};
  const f32x2v q0 = g0 * fma2((f32x2v)-0.5f, a0, (f32x2v)1.0f), q1 = g1 * fma2((f32x2v)-0.5f, a1, (f32x2v)1.0f);
  const f32x2v n0 = (0.5f * g0) * a0, n1 = (0.5f * g1) * a1;
  g0 = (f32x2v){x0.x >= 0.f ? q0.x : n0.x, x0.y >= 0.f ? q0.y : n0.y};
  g1 = (f32x2v){x1.x >= 0.f ? q1.x : n1.x, x1.y >= 0.f ? q1.y : n1.y};
}
"""),
        ("""          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = acc[mi][ni][r] * gelu_erf(acc[mi][ni + 2][r]);
          pk[ni] = uint2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};""",
         """          f32x2v g0 = (f32x2v){acc[mi][ni + 2][0], acc[mi][ni + 2][1]};
          f32x2v g1 = (f32x2v){acc[mi][ni + 2][2], acc[mi][ni + 2][3]};
          gelu_erf2x2(g0, g1);
          const f32x2v o0 = (f32x2v){acc[mi][ni][0], acc[mi][ni][1]} * g0;
          const f32x2v o1 = (f32x2v){acc[mi][ni][2], acc[mi][ni][3]} * g1;
          pk[ni] = uint2{pack_bf16x2(o0.x, o0.y), pack_bf16x2(o1.x, o1.y)};"""),
    ],
    "noprio": [
        ("  __builtin_amdgcn_s_setprio(1);                       \\\n  mma(QM, NI, FB);                                     \\\n"
         "  __builtin_amdgcn_s_setprio(0);                       \\\n",
         "  mma(QM, NI, FB);                                     \\\n"),
    ],
}


# variants whose launch swaps need the lab kernels patched back into the copy
OVERLAY = {"mf32": "lab_kernels.patch", "w4": "lab_kernels.patch"}


def main():
    name = sys.argv[1]
    build = OUT / "build"
    build.mkdir(exist_ok=True)
    src = (CSRC / "gemm.hip").read_text()
    if name in OVERLAY:
        base = build / f"gemm_{name}_base.hip"
        base.write_text(src)
        subprocess.run(["patch", "-s", str(base), str(OUT / "patches" / OVERLAY[name])], check=True)
        src = base.read_text()
    for old, new in VARIANTS[name]:
        assert src.count(old) == 1, old
        src = src.replace(old, new)
    (build / f"gemm_{name}.hip").write_text(src)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I", str(CSRC), "-c",
                    str(build / f"gemm_{name}.hip"), "-o", str(build / f"gemm_{name}.o")], check=True)
    objs = [str(p) for p in sorted((CSRC / "build").glob("*.o")) if p.name != "gemm.o"]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", str(build / f"gemm_{name}.o"),
                    *objs, "-o", str(OUT / f"libnewsrec_{name}.so")], check=True)
    print("built", name)


if __name__ == "__main__":
    sys.exit(main())
