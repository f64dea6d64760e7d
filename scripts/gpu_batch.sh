set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 8 16; do
timeout -k 10 300 python bench.py --batch_size $b --steps 6 --warmup 2 --profile > gpurun_out/llama_b$b.log 2>&1 || exit 1
done
