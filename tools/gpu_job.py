#!/usr/bin/env python3
"""One parametrised runner for GPU-box jobs (replaces the per-experiment shell scripts).

    gpurun --timeout 900 -- python tools/gpu_job.py tests smoke bench
    gpurun -- python tools/gpu_job.py bench --set batch=32 --tag b32
    gpurun -- python tools/gpu_job.py prof --set preset=gpt2_774m_ddp

Each recipe is a list of steps; every step runs under its own ``timeout -k 10 <s>``, its output
goes to ``gpurun_out/<tag>/<step>.log`` and is streamed to stdout as it comes (so a long step
shows progress), and the first failing step ends the job with its exit status — nothing else
runs on the GPU after a failure, a timeout or a crash.
"""
from __future__ import annotations

import argparse
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable


def _bench(extra="", steps=10, warmup=3):
    return f"{PY} -u bench.py --steps {steps} --warmup {warmup} {extra}".strip()


def recipes(p):
    """name -> [(step, timeout_s, command)]; ``p`` holds the --set overrides."""
    pre = f"--preset {p['preset']} " if p.get("preset") else ""
    bs = f"--batch_size {p['batch']} " if p.get("batch") else ""
    ck = f"--actv_ckpt {p['ckpt']} " if p.get("ckpt") else ""
    extra = pre + bs + ck + p.get("args", "")
    steps = int(p.get("steps", 10))
    return {
        "tests": [("gpu_tests", 900, f"{PY} -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "
                   "-p no:cacheprovider " + p.get("tests", ""))],
        "smoke": [("smoke", 300, f"{PY} -u -c 'import __graft_entry__ as g; g.smoke()'")],
        "bench": [("bench", 600, _bench(extra, steps))],
        "presets": [(f"preset_{n}", 500, _bench(f"--preset {n} " + p.get("args", ""), steps))
                    for n in ("llama3_8b_fsdp", "gpt2_774m_ddp", "llama32_1b_lora_alpaca", "llama2_7b_fsdp_mp")],
        "prof": [("prof", 600, f"rocprofv3 --kernel-trace --stats -d gpurun_out/{p['tag']}/rocprof -o run -- "
                  + _bench(extra, int(p.get("steps", 3)), 2)),
                 ("breakdown", 120, f"{PY} tools/step_breakdown.py \"$(find gpurun_out/{p['tag']}/rocprof -name "
                  f"'*.db' -print -quit)\" --marker {p.get('marker', 'emb_fwd')}"),
                 ("kstats", 120, f"{PY} tools/kstats.py \"$(find gpurun_out/{p['tag']}/rocprof -name "
                  f"'*.db' -print -quit)\" --grep '{p.get('kgrep', '')}'"),
                 # the trace database is tens of MiB: drop it so gpurun_out/ stays under the copy-back cap
                 ("cleanup", 60, f"rm -rf gpurun_out/{p['tag']}/rocprof")],
        "cmd": [("cmd", int(p.get("timeout", 600)), p.get("cmd", "true"))],
    }


def run_step(name, tmo, cmd, outdir):
    log = os.path.join(outdir, f"{name}.log")
    print(f"[gpu_job] {name}: {cmd}  (limit {tmo}s, log {log})", flush=True)
    t0 = time.time()
    with open(log, "w") as f:
        pr = subprocess.Popen(["timeout", "-k", "10", str(tmo), "bash", "-o", "pipefail", "-c", cmd], cwd=ROOT,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, bufsize=1)
        for line in pr.stdout:
            f.write(line)
            f.flush()
            sys.stdout.write(line)
            sys.stdout.flush()
        rc = pr.wait()
    print(f"[gpu_job] {name}: rc={rc} in {time.time() - t0:.0f}s", flush=True)
    return rc


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("recipes", nargs="+")
    ap.add_argument("--set", action="append", default=[], help="key=value recipe parameter")
    ap.add_argument("--tag", default=None)
    a = ap.parse_args(argv)
    p = dict(kv.split("=", 1) for kv in a.set)
    p["tag"] = a.tag or "_".join(a.recipes)
    outdir = os.path.join(ROOT, "gpurun_out", p["tag"])
    os.makedirs(outdir, exist_ok=True)
    os.environ.setdefault("TMPDIR", "/tmp")
    book = recipes(p)
    for r in a.recipes:
        if r not in book:
            raise SystemExit(f"unknown recipe {r!r}; known: {sorted(book)}")
    for r in a.recipes:
        for name, tmo, cmd in book[r]:
            rc = run_step(name, tmo, cmd, outdir)
            if rc != 0:
                print(f"[gpu_job] stopping after {name} (rc={rc})", flush=True)
                return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
