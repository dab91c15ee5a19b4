set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for b in 128 256; do
  timeout -k 10 300 python -u bench.py --workload mistral --batch $b > gpurun_out/r2_mistral_b$b.log 2>&1 || exit $?
  echo "== mistral b$b"; tail -1 gpurun_out/r2_mistral_b$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'])"
done
for b in 48 64; do
  SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_sd_b$b.json timeout -k 10 400 python -u bench.py --batch $b --steps 3 --warmup 1 --latency-runs 1 > gpurun_out/r2_sd_b$b.log 2>&1 || exit $?
  echo "== sd b$b"; tail -1 gpurun_out/r2_sd_b$b.log | cut -c1-200
done
