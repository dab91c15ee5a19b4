#!/bin/bash
# Round 5 evidence: rocprofv3 kernel traces of Flux 512^2 / 1024^2 (one timed generate after warm-up) and of SD2.1
# batch-1 (latency regime), summarised with tools/prof_db.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for res in 512 1024; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5r_flux$res -o run -- python3 -u bench.py --workload flux \
    --height $res --width $res --steps 1 --warmup 1 --inference-steps 28 --latency-runs 0 > gpurun_out/r5r_flux$res.log 2>&1 || { tail -20 gpurun_out/r5r_flux$res.log; exit 1; }
  tail -1 gpurun_out/r5r_flux$res.log | cut -c1-200
  python3 tools/prof_db.py $(find gpurun_out/r5r_flux$res -name "*results.db" | head -1) --top 30 \
    --title "Flux.1-dev $res^2, 28 steps (round 5)" > gpurun_out/r5r_flux$res.md && rm -rf gpurun_out/r5r_flux$res
done
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5r_sdb1 -o run -- python3 -u bench.py --batch 1 --steps 2 --warmup 1 \
  --latency-runs 0 > gpurun_out/r5r_sdb1.log 2>&1 || { tail -20 gpurun_out/r5r_sdb1.log; exit 1; }
tail -1 gpurun_out/r5r_sdb1.log | cut -c1-200
python3 tools/prof_db.py $(find gpurun_out/r5r_sdb1 -name "*results.db" | head -1) --top 40 \
  --title "SD2.1 batch 1 (round 5)" > gpurun_out/r5r_sdb1.md && rm -rf gpurun_out/r5r_sdb1
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5r_vit -o run -- python3 -u bench.py --workload vit --steps 20 --warmup 3 \
  > gpurun_out/r5r_vit.log 2>&1 || { tail -20 gpurun_out/r5r_vit.log; exit 1; }
tail -1 gpurun_out/r5r_vit.log | cut -c1-200
python3 tools/prof_db.py $(find gpurun_out/r5r_vit -name "*results.db" | head -1) --top 30 \
  --title "ViT-base/16 batch 32 (round 5)" > gpurun_out/r5r_vit.md && rm -rf gpurun_out/r5r_vit
