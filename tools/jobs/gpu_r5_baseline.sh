# Round-5 baseline on one box: headline bench exactly as the driver runs it (20 timed, 5 warm-up)
# with the new telemetry fields, then the forward-layout GEMM A/B (ours vs hipBLASLt).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r5base
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5base/bench.log 2>&1 || { tail -30 gpurun_out/r5base/bench.log; exit 3; }
tail -1 gpurun_out/r5base/bench.log
timeout -k 10 300 python -u tools/bench_gemm_nt.py --rounds 3 > gpurun_out/r5base/gemm_nt.jsonl 2>&1 || { tail -20 gpurun_out/r5base/gemm_nt.jsonl; exit 4; }
cat gpurun_out/r5base/gemm_nt.jsonl
