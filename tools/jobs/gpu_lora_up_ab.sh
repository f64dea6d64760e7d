# lora_up with its t rows prefetched a tile ahead: numerics, then the microbench new vs previous
# build (the previous .so swapped in on the box's scratch copy; needs
# building_llm_from_scratch_amd/_C_prev.so, the previous build, copied in by hand for the run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/loraup; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_model_gpu.py -k "lora" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 120 python -u tools/bench_lora.py --only up > $O/new_$r.jsonl 2>&1 || exit 4
  cp building_llm_from_scratch_amd/_C.so /tmp/_C_new.so && cp building_llm_from_scratch_amd/_C_prev.so building_llm_from_scratch_amd/_C.so
  timeout -k 10 120 python -u tools/bench_lora.py --only up > $O/prev_$r.jsonl 2>&1 || exit 5
  cp /tmp/_C_new.so building_llm_from_scratch_amd/_C.so
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/loraup/*.jsonl")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f.split("/")[-1], d["group"], {k: v["us"] for k, v in d.items() if isinstance(v, dict)})
PY
