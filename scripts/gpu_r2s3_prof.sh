# Round-2 session 3: rocprof breakdown of the headline (recompute SwiGLU + RoPE-bwd fusions), LoRA and GPT-2 presets
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/p9
cd /tmp && export TMPDIR=/tmp
for cfg in llama:"" lora:"--preset llama32_1b_lora_alpaca" gpt2:"--preset gpt2_774m_ddp"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/p9_$name -o run -- python3 $R/bench.py $args --steps 2 --warmup 2 > $R/gpurun_out/p9/$name.log 2>&1 || { tail -20 $R/gpurun_out/p9/$name.log; exit 1; }
  python3 $R/tools/step_breakdown.py /tmp/p9_$name/run_results.db > $R/gpurun_out/p9/${name}_breakdown.md 2>&1
  python3 $R/tools/rocpd_summary.py /tmp/p9_$name/run_results.db --top 40 --md $R/gpurun_out/p9/${name}_top.md > /dev/null 2>&1
  head -24 $R/gpurun_out/p9/${name}_breakdown.md
done
