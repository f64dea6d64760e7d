# Same-box A/B: activation-checkpoint mode none vs selective at the bench config.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --actv_ckpt none > gpurun_out/ckpt_none.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ckpt_sel.log 2>&1
