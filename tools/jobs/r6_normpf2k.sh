# norm backward prefetch at d = 2048 (Llama-3.2-1B RMSNorm, 4 waves x 1 vector): shipped rule
# (prefetch below 4 waves) vs _C_v.so (prefetch for every single-vector row), ABAB, kernel only
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6normpf2k
P=building_llm_from_scratch_amd
cp $P/_C.so /tmp/_C_base.so
for arm in base v base v; do
  if [ "$arm" = v ]; then cp $P/_C_v.so $P/_C.so; else cp /tmp/_C_base.so $P/_C.so; fi
  timeout -k 10 120 python -u -c "
import torch, sys, json; sys.path.insert(0, '.')
from building_llm_from_scratch_amd import ops
ops.load_ext(required=True)
def timeit(fn, iters=30):
    for _ in range(3): fn()
    torch.cuda.synchronize(); s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e) / iters * 1e3
out = {}
for N, d in ((32768, 2048), (98304, 2048)):
    x = torch.randn(N, d, device='cuda').to(torch.bfloat16); dy = torch.randn_like(x); acc = torch.randn_like(x)
    w = torch.randn(d, device='cuda').to(torch.bfloat16)
    _, rstd = ops.rmsnorm_fwd(x, w, 1e-5)
    t = timeit(lambda: ops.rmsnorm_bwd(dy, x, w, rstd, dx_acc=acc))
    out[f'rms_{N}x{d}'] = {'us': round(t, 1), 'TBps': round(4 * N * d * 2 / t / 1e6, 2)}
print(json.dumps(out))
" > gpurun_out/r6normpf2k/$arm.json 2>&1 || { tail -20 gpurun_out/r6normpf2k/$arm.json; exit 5; }
  echo "$arm $(tail -1 gpurun_out/r6normpf2k/$arm.json)"
done
cp /tmp/_C_base.so $P/_C.so
