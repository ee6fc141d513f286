#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of the pool+score kernel into
profiles/pmc_pool_score.json (read by bench.py for roofline.traffic).

HBM/fabric bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of a
wide (16 B/lane) coalesced read, so read bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE is exact for 16-B stores (the score stores here are 4 B/lane,
uncalibrated, and < 0.2 % of the traffic).  Infinity-Cache hits are counted
by these memory-side counters, so this is traffic beyond L2.

    python tools/pmc_summary.py gpurun_out/prof_r1 profiles/pmc_pool_score.json
"""
import csv
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def counters(d: Path):
    out = {}
    for r in csv.DictReader(open(d / "pmc_counter_collection.csv")):
        out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in out.items()}


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    import bench
    from news_recommendation_project_v2_amd import synthetic
    imps = synthetic.mind_shaped("mind_large_dev", seed=1234)
    res = json.loads(dst.read_text()) if dst.exists() else {}  # configs not in `src` keep their last values
    for cfg in ("latent_bf16", "final_bf16", "latent_fp32"):
        pooler, dt = cfg.split("_")
        if not (src / f"pmc_{cfg}_FETCH_SIZE").is_dir():
            continue
        f = counters(src / f"pmc_{cfg}_FETCH_SIZE")["FETCH_SIZE"]
        w = counters(src / f"pmc_{cfg}_WRITE_SIZE")["WRITE_SIZE"]
        hm = counters(src / f"pmc_{cfg}_TCC_HIT_sum_TCC_MISS_sum")
        alg = bench.ps_bytes(imps, pooler, 2 if dt == "bf16" else 4)
        traffic = 2 * f * 1024 + w * 1024
        res[cfg] = round(traffic)
        res[cfg + "_detail"] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "read_bytes_corrected": 2 * f * 1024,
                                "write_bytes": w * 1024, "algorithmic_bytes": alg,
                                "traffic_over_algorithmic": round(traffic / alg, 4),
                                "L2_hit_rate": round(hm["TCC_HIT_sum"] / (hm["TCC_HIT_sum"] + hm["TCC_MISS_sum"]), 4)}
    dst.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
