#!/bin/bash
# Round 3 (end): SD2.1 breaking point re-measured on the final kernels with STEP-LEVEL batching (requests join the running batch at the next denoising step), the reference's own metric (find-compute-breaking-point.yaml:21-56,
# README.md:125): the real SD2.1 server (random-init weights, step-level batching up to 16 rows) on 127.0.0.1:8000,
# closed-loop clients calling GET /load/1/infer/50 (one 512x512 image, 50 DDIM steps per request), ramped until
# the p50 latency passes 900 ms or throughput plateaus.  The server is started here and stopped by its PID.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAI_SD_MAX_BATCH=16 PORT=8000 HOST=127.0.0.1 NUM_OF_RUNS_INF=50 timeout -k 10 900 python -u -c "import shai_amd.serving.sd as m; m.main()" > gpurun_out/bp_server.log 2>&1 &
SRV=$!
ok=0
for i in $(seq 1 300); do
  [ $((i % 20)) -eq 0 ] && echo "waiting for the server ($i polls)"
  if python - <<'PY' 2>/dev/null
import urllib.request, sys
sys.exit(0 if urllib.request.urlopen("http://127.0.0.1:8000/readiness", timeout=2).status == 200 else 1)
PY
  then ok=1; break; fi
  kill -0 $SRV 2>/dev/null || break
  sleep 2
done
if [ $ok -ne 1 ]; then echo "server not ready"; tail -20 gpurun_out/bp_server.log; kill $SRV 2>/dev/null; exit 1; fi
echo "server ready after ${i} polls"
timeout -k 10 700 python -u - > gpurun_out/bp_result.json <<'PY'
import json, sys
sys.path.insert(0, ".")
import shai_amd  # noqa: F401
from shai_amd.bench.client import run_clients
from shai_amd.bench.breaking_point import find_breaking_point
url = "http://127.0.0.1:8000/load/1/infer/50"
warm = run_clients(8, url, 15.0).summary()           # (the server captured every batch bucket at start-up)
res = find_breaking_point(url, step_s=60.0, clients_seq=[2, 4, 6, 7, 8, 10])
res["warmup"] = warm
res["request"] = "GET /load/1/infer/50 (1 image, 512x512, 50 DDIM steps, CFG 7.5)"
print(json.dumps(res, indent=1))
PY
rc=$?
kill $SRV 2>/dev/null
wait $SRV 2>/dev/null
[ $rc -eq 0 ] || { tail -20 gpurun_out/bp_result.json; exit $rc; }
python -c "
import json; r = json.load(open('gpurun_out/bp_result.json'))
print('breaking point:', json.dumps(r['breaking_point']), 'per min:', r['throughput_per_min'])
for s in r['steps']: print(s)"
