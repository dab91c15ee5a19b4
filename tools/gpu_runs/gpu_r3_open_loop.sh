#!/bin/bash
# Open-loop (Poisson) SD2.1 latency on one MI355X: the real server with step-level batching vs request-level
# batching (SHAI_SD_STEP_BATCHING=0), GET /load/1/infer/50 arriving at 3 and 6 requests/s for 60 s each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for mode in 1 0; do
  SHAI_SD_STEP_BATCHING=$mode SHAI_SD_MAX_BATCH=16 PORT=8000 HOST=127.0.0.1 NUM_OF_RUNS_INF=50 timeout -k 10 600 \
    python -u -c "import shai_amd.serving.sd as m; m.main()" > gpurun_out/ol_server_$mode.log 2>&1 &
  SRV=$!
  ok=0
  for i in $(seq 1 300); do
    [ $((i % 20)) -eq 0 ] && echo "waiting for the server ($i polls)"
    if python -c "import urllib.request, sys; sys.exit(0 if urllib.request.urlopen('http://127.0.0.1:8000/readiness', timeout=2).status == 200 else 1)" 2>/dev/null; then ok=1; break; fi
    kill -0 $SRV 2>/dev/null || break
    sleep 2
  done
  if [ $ok -ne 1 ]; then echo "server not ready"; tail -20 gpurun_out/ol_server_$mode.log; kill $SRV 2>/dev/null; exit 1; fi
  timeout -k 10 300 python -u - $mode > gpurun_out/ol_result_$mode.json <<'PY'
import json, sys
sys.path.insert(0, ".")
import shai_amd  # noqa: F401
from shai_amd.bench.client import run_clients, run_open_loop
url = "http://127.0.0.1:8000/load/1/infer/50"
run_clients(6, url, 10.0)   # warm
out = {"step_batching": sys.argv[1] == "1", "request": "GET /load/1/infer/50 (512x512, 50 DDIM steps)"}
for rate in (3.0, 6.0):
    out[f"poisson_{rate:g}rps"] = run_open_loop(rate, url, 60.0, seed=7).summary()
print(json.dumps(out))
PY
  rc=$?
  kill $SRV 2>/dev/null; wait $SRV 2>/dev/null
  [ $rc -eq 0 ] || { tail -5 gpurun_out/ol_result_$mode.json; exit $rc; }
  echo "== step_batching=$mode"; cat gpurun_out/ol_result_$mode.json
done
