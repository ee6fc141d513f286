"""scripts/eval.py over 2 and 4 ranks (BASELINE config 4 path: impressions partitioned
by cost, news-table transform sharded and all-gathered, scores gathered back)
gives exactly the single-rank per-candidate scores (bit for bit), dense ranks and
metrics.  The ranks run with the gloo backend and
share the test box's one GPU (RCCL needs one GPU per rank; the 8-GPU RCCL run is
the driver's multi-GPU bench), so this checks the partitioning, the sharded
transform + gather and the score reassembly, not the xGMI transport."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _last_record(d: Path) -> dict:
    return json.loads((d / "final_scores.jsonl").read_text().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("pooler,ranks", [("final", 2), ("latent", 2), ("latent", 4)])
def test_eval_two_ranks_matches_one(tmp_path, pooler, ranks):
    env = dict(os.environ, NR_DIST_BACKEND="gloo", PYTHONPATH=str(REPO), OMP_NUM_THREADS="4")
    args = ["scripts/eval.py", "--synthetic", "--num-impressions", "700", "--splits", "MINDsmall_dev",
            "--pooler", pooler]
    one = subprocess.run([sys.executable, *args, "--log-dir", str(tmp_path / "one"), "--dump-scores",
                          str(tmp_path / "one")], cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert one.returncode == 0, one.stderr[-3000:]
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
                          "--master-addr", "127.0.0.1", "--master-port", str(_port()), *args,
                          "--log-dir", str(tmp_path / "two"), "--dump-scores", str(tmp_path / "two")], cwd=REPO,
                         env=env, capture_output=True, text=True, timeout=240)
    assert two.returncode == 0, two.stderr[-3000:]
    a, b = _last_record(tmp_path / "one"), _last_record(tmp_path / "two")
    assert a["val_scores"] == b["val_scores"]
    assert a["val_scores"]["num_samples"] > 0
    # per candidate, not only the means: a misplaced all-gather chunk or a reassembly
    # permutation that preserves the averages would show here
    for split in ("MINDsmall_dev",):
        s1, s2 = np.load(tmp_path / "one" / f"{split}.npz"), np.load(tmp_path / "two" / f"{split}.npz")
        assert s1["scores"].shape == s2["scores"].shape and len(s1["scores"]) > 0
        assert np.array_equal(s1["scores"].view(np.uint32), s2["scores"].view(np.uint32))
        assert np.array_equal(s1["ranks"], s2["ranks"])
