# Round-2: decode (sample print) speed.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for M in "llama3 8B" "GPT2 774M" "GPT2 124M" "llama3_2 1B"; do
  set -- $M
  timeout -k 10 200 python tools/bench_decode.py --model $1 --num_params $2 >> gpurun_out/r2_decode.log 2>&1 || exit 1
done
