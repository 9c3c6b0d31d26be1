#!/bin/bash
# GPU-box step for round-3 iterations: selected parity tests, then the bench (each step under
# its own time limit; stop at the first failure).  PYTEST_K selects tests, BENCH_ARGS / TAG
# the bench run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    -k "$PYTEST_K" > gpurun_out/pytest_${TAG}.log 2>&1
  rc=$?
  tail -4 gpurun_out/pytest_${TAG}.log
  [ $rc = 0 ] || exit $rc
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 500 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
  rc=$?
  tail -3 gpurun_out/bench_${TAG}.err
  [ $rc = 0 ] || exit $rc
  python3 - gpurun_out/bench_${TAG}.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"], "ms", d["ms_per_step"], "ratio", d["compression_ratio"], "ok", d["roundtrip_ok"])
print("kernels", json.dumps(d["kernels"]))
for k in ("frontend", "h2d_d2h", "recordbatch", "zstd", "deflate", "deflate_dynamic", "secondary"):
    if k in d:
        v = d[k]
        print(k, json.dumps({a: v[a] for a in v if a in ("value", "ms_per_step", "ms_per_roundtrip", "overhead_vs_c_abi", "roundtrip_ok", "kernels", "compress_call_ms", "decompress_call_ms", "recycle_call_ms", "roundtrip_gibs", "link_h2d_gibs", "link_d2h_gibs", "decompress_gibs")}))
if "stock_decode" in d:
    print("stock", json.dumps({k: v["avg_launch_ms"] for k, v in d["stock_decode"].items()}))
PY
fi
