# end-to-end same-box ABAB: this tree's extension (round-6 attention changes: XCD order, 16-B
# backward stores, dropout fold) vs _C_before.so (built from commit 621bfe1), headline + GPT-2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6e2e
P=building_llm_from_scratch_amd
cp $P/_C.so /tmp/_C_after.so
for arm in after before after before; do
  if [ "$arm" = before ]; then cp $P/_C_before.so $P/_C.so; else cp /tmp/_C_after.so $P/_C.so; fi
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6e2e/hl_$arm.log 2>&1 || { tail -20 gpurun_out/r6e2e/hl_$arm.log; exit 5; }
  echo "headline $arm $(tail -1 gpurun_out/r6e2e/hl_$arm.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --preset gpt2_774m_ddp > gpurun_out/r6e2e/g2_$arm.log 2>&1 || { tail -20 gpurun_out/r6e2e/g2_$arm.log; exit 6; }
  echo "gpt2 $arm $(tail -1 gpurun_out/r6e2e/g2_$arm.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
done
cp /tmp/_C_after.so $P/_C.so
