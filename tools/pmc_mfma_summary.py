#!/usr/bin/env python3
"""Summarise the MFMA-busy PMC passes of tools/profile_round2.sh (persistent
GEMM shapes and the encoder attention_kernel) into one JSON.

Per kernel (medians over its dispatches):
  mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (cycles * 4 SIMDs * CUs), where
    cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs) and
    SQ_VALU_MFMA_BUSY_CYCLES = 16 * SQ_INSTS_MFMA for v_mfma_f32_16x16x32_bf16
    (checked below: mfma_busy_per_inst);
  clock_GHz from the kernel-trace duration when given;
  read bytes beyond L2 = 2 * FETCH_SIZE KiB (gfx950 halves wide reads,
    MI355X_MICROARCH.md §HBM; Infinity-Cache hits included).

    python tools/pmc_mfma_summary.py gpurun_out/prof_r2 profiles/round2/pmc_mfma.json
"""
import csv
import glob
import json
import statistics
import sys
from pathlib import Path

CUS = 256


def passes(d: Path):
    out = {}
    for p in sorted(glob.glob(str(d / "p*" / "pmc_counter_collection.csv"))):
        for r in csv.DictReader(open(p)):
            out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in out.items()}


def kernel_ms(trace_csv: Path, needle: str):
    if not trace_csv.exists():
        return None
    for r in csv.DictReader(open(trace_csv)):
        if needle in r["Name"]:
            return float(r["AverageNs"]) / 1e6
    return None


def summarise(c: dict, ms):
    cycles = c["GRBM_GUI_ACTIVE"] / 8
    res = {
        "SQ_INSTS_MFMA": c["SQ_INSTS_MFMA"],
        "SQ_VALU_MFMA_BUSY_CYCLES": c["SQ_VALU_MFMA_BUSY_CYCLES"],
        "SQ_BUSY_CYCLES": c["SQ_BUSY_CYCLES"],
        "GRBM_GUI_ACTIVE": c["GRBM_GUI_ACTIVE"],
        "kernel_cycles": cycles,
        "mfma_busy_per_inst": c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(c["SQ_INSTS_MFMA"], 1),
        "mfma_busy_frac": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cycles * 4 * CUS),
        "wave_cycles_waiting_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
        "wave_cycles_issue_stall_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
        "lds_bank_conflict_per_lds_inst": c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_INSTS_LDS"], 1),
        "L2_hit_rate": c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]),
        "read_bytes_beyond_L2": 2 * c["FETCH_SIZE"] * 1024,
    }
    if ms:
        res["kernel_ms_trace"] = ms
        res["clock_GHz"] = cycles / (ms * 1e-3) / 1e9
    return res


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    out = {}
    for d in sorted(src.glob("gemm_*")):
        c = passes(d)
        # M = 72,023 rows padded to 282 tiles of 256; flops = 2 M N K
        n, k = int(d.name.split("_")[1][1:]), int(d.name.split("_")[2][1:])
        r = summarise(c, None)
        r["flop"] = 2.0 * 72023 * n * k
        r["expected_mfma_insts"] = 282 * 256 * n * k / (16 * 16 * 32)
        out[d.name] = r
    if (src / "attention").exists():
        out["attention_kernel_bf16"] = summarise(passes(src / "attention"), None)
        out["attention_kernel_bf16"]["note"] = ("encoder_bench --n-news 4096 (titles ~20 tokens): per-dispatch medians "
                                                "over the 24 layers x 2 reps; short sequences keep the MFMA share low")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
