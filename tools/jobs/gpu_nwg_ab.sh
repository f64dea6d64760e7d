# TEMPORARY A/B of the norm-backward workgroup cap (BLLM_EXP_NWG) on the elementwise bench shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/nwg
for n in 1024 2048 4096 512; do
BLLM_EXP_NWG=$n timeout -k 10 120 python tools/bench_ew.py > gpurun_out/nwg/ew_$n.json 2>&1 || exit 3
echo "$n $(python -c "import json;d=json.loads(open('gpurun_out/nwg/ew_$n.json').read().strip().splitlines()[-1]);print({k:v['us'] for k,v in d.items() if 'norm' in k})")"
done
