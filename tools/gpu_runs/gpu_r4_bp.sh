#!/bin/bash
# Round 4: SD2.1 breaking point with the reference's 300 s holds (find-compute-breaking-point.yaml:24-25,47-52),
# split over gpurun calls (each call is capped at 20 min: server start-up + at most 3 holds).
#   bash tools/gpu_runs/gpu_r4_bp.sh "1,2,4" a      -> gpurun_out/bp300_a.json
# The real SD2.1 server (random-init weights, step-level batching up to 16 rows) on 127.0.0.1:8000; closed-loop
# clients call GET /load/1/infer/50 (one 512x512 image, 50 DDIM steps).  A hold's line is printed as it completes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CLIENTS=$1
TAG=$2
SHAI_SD_MAX_BATCH=16 PORT=8000 HOST=127.0.0.1 NUM_OF_RUNS_INF=50 timeout -k 10 1140 python -u -c "import shai_amd.serving.sd as m; m.main()" > gpurun_out/bp300_server_$TAG.log 2>&1 &
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
if [ $ok -ne 1 ]; then echo "server not ready"; tail -20 gpurun_out/bp300_server_$TAG.log; kill $SRV 2>/dev/null; exit 1; fi
echo "server ready after ${i} polls"
timeout -k 10 1000 python -u - "$CLIENTS" "$TAG" <<'PY'
import json, sys
sys.path.insert(0, ".")
import shai_amd  # noqa: F401
from shai_amd.bench.client import run_clients
from shai_amd.bench.breaking_point import find_breaking_point
url = "http://127.0.0.1:8000/load/1/infer/50"
seq = [int(c) for c in sys.argv[1].split(",")]
warm = run_clients(4, url, 10.0).summary()
out = f"gpurun_out/bp300_{sys.argv[2]}.json"
def on_step(s):
    print("step", json.dumps(s), flush=True)
res = find_breaking_point(url, step_s=300.0, clients_seq=seq, progress_s=60.0, on_step=on_step)
res["warmup"] = warm
res["hold_s"] = 300.0
res["request"] = "GET /load/1/infer/50 (1 image, 512x512, 50 DDIM steps, CFG 7.5)"
json.dump(res, open(out, "w"), indent=1)
print("breaking point:", json.dumps(res["breaking_point"]), "per min:", res["throughput_per_min"])
PY
rc=$?
kill $SRV 2>/dev/null
wait $SRV 2>/dev/null
exit $rc
