#!/bin/bash
# round-6 batch 7: the exact lines the driver's scaling run will parse, rehearsed on one GPU (gloo:
# the ranks share the card, so the values are not scaling numbers; the structure, the checks and
# every component are): python bench.py --gpus N --steps 20 --warmup 5 for N = 2, 4, 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp PLK_DIST_BACKEND=gloo MASTER_ADDR=127.0.0.1
for n in 2 4 8; do
  timeout -k 10 420 python -u bench.py --gpus $n --steps 20 --warmup 5 > $O/b7_bench_n$n.json 2> $O/b7_bench_n$n.err \
    || { echo "N=$n failed"; tail -30 $O/b7_bench_n$n.err; exit 1; }
  python3 - $O/b7_bench_n$n.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c = d["components"]
print(d["n_gpus"], d["scaling"], d["config"]["points_per_gpu"], d["checks"], sorted(c)[:40])
print("  replicas", {k: c["prove_2^20_gates_replicas"][k] for k in ("gpus", "matches_oracle_all_ranks", "deterministic_all_ranks")},
      "split", {k: c["prove_2^20_gates_split"][k] for k in ("gpus", "matches_oracle", "same_as_single_gpu")})
PY
done
