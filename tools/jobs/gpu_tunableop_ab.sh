set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/tune
timeout -k 10 600 python -u bench.py --preset gpt2_774m_ddp --steps 2 --warmup 1 --tunableop_tune gpurun_out/tune/gpt2.csv > gpurun_out/tune/tune_gpt2.log 2>&1 || exit 3
ls gpurun_out/tune
for i in 1 2; do
timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 > gpurun_out/tune/base_$i.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 --tunableop gpurun_out/tune/gpt20.csv > gpurun_out/tune/tuned_$i.log 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/tune/hl_base_$i.log 2>&1 || exit 6
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --tunableop configs/tunableop_llama3_8b_b40_mi355x.csv > gpurun_out/tune/hl_tuned_$i.log 2>&1 || exit 7
done
grep -ho '"value": [0-9.]*' gpurun_out/tune/*.log
