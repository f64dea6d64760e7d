# dW GEMM tile -> XCD map / group depth A/B (same process, interleaved; hipBLASLt as control)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/wgmap
V="map1:BLLM_WG_MAP=1;map2:BLLM_WG_MAP=2;gm4:BLLM_WG_GM=4;gm16:BLLM_WG_GM=16;map2gm4:BLLM_WG_MAP=2,BLLM_WG_GM=4;map2gm16:BLLM_WG_MAP=2,BLLM_WG_GM=16"
timeout -k 10 400 python -u tools/bench_wgrad.py --tokens 40960 --models llama3_8b --rounds 3 --variants "$V" > gpurun_out/wgmap/llama.jsonl 2>&1 || { tail -5 gpurun_out/wgmap/llama.jsonl; exit 3; }
timeout -k 10 300 python -u tools/bench_wgrad.py --tokens 65536 --models gpt2_774m --rounds 3 --variants "$V" > gpurun_out/wgmap/gpt2.jsonl 2>&1 || { tail -5 gpurun_out/wgmap/gpt2.jsonl; exit 4; }
python3 - <<'PY'
import json
for f in ("gpurun_out/wgmap/llama.jsonl", "gpurun_out/wgmap/gpt2.jsonl"):
    for l in open(f):
        if not l.startswith("{"): continue
        r = json.loads(l)
        print(r["model"], r["gemm"], r["auto_splits"], {k[:-7]: v for k, v in r.items() if k.endswith("_tflops")})
PY
