# round 6: the module-API training tests (exact-norm clip on the oracle side), the API
# end-to-end test and the host-logic tests on the box, then the API leg of the bench
set -o pipefail
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_latent_attention_autograd.py tests/test_final_attention_autograd.py tests/test_api_end_to_end.py \
  tests/test_host_logic.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u - > $O/api.json 2> $O/api.err <<'PY'
import json, sys
sys.path.insert(0, ".")
import torch
import bench
from news_recommendation_project_v2_amd import synthetic
dev = torch.device("cuda", 0)
n_news, n_imp = synthetic.SHAPES["mind_large_dev"]
imps = synthetic.mind_impressions(n_news, n_imp, seed=1234)
table = bench.news_table(n_news, dev).cpu()
print(json.dumps(bench.api_end_to_end("latent", "bf16", imps, table, dev)))
PY
