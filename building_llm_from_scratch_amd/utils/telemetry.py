"""Device telemetry for benchmark lines: what the GPU's clocks, power, temperature and throttle
state were while a timed region ran, plus the library versions the GEMM tuning depends on.

Two boxes running the same tree can differ by a few percent in tokens/s (the driver's round-4
headline was 2.8 % under the builder's own runs).  The bench JSON therefore carries, for the
timed loop only:

* the average / min graphics clock (SCLK, over every XCD) and memory clock (MCLK) sampled every
  ``interval`` seconds from the SMU metrics table (``amdsmi_get_gpu_metrics_info``: the same
  numbers ``amd-smi metric`` prints; AMD SMI reads the driver, it does not initialise HIP);
* average / max socket power, max hotspot and HBM temperature;
* the fraction of the region the firmware spent under the power limit (PPT), the socket
  thermal limit and PROCHOT, from the residency accumulators' deltas over the accumulation
  counter; and the xGMI read / write byte accumulators' deltas (what the links moved).

Everything is best effort: on a CPU box, or when the metrics table lacks a field, the value
is ``None`` — never an exception in the bench.
"""
from __future__ import annotations

import os
import threading
from typing import Any, Dict, List, Optional

_NA = (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF)


def _num(v) -> Optional[float]:
    if isinstance(v, (list, tuple)):
        vals = [float(x) for x in v if isinstance(x, (int, float)) and x not in _NA and x > 0]
        return sum(vals) / len(vals) if vals else None
    if isinstance(v, (int, float)) and v not in _NA:
        return float(v)
    return None


def _amdsmi_handle(local_rank: int = 0):
    """(amdsmi module, processor handle) of this rank's GPU, or (None, None)."""
    try:
        import amdsmi
        amdsmi.amdsmi_init()
        handles = amdsmi.amdsmi_get_processor_handles()
    except Exception:
        return None, None
    if not handles:
        return None, None
    # HIP's visible-device list, when set, picks which physical GPU this rank is
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") \
        or os.environ.get("CUDA_VISIBLE_DEVICES")
    idx = local_rank
    if vis:
        ids = [s for s in vis.split(",") if s.strip()]
        if local_rank < len(ids) and ids[local_rank].strip().isdigit():
            idx = int(ids[local_rank])
    if len(handles) == 1:
        idx = 0
    if idx >= len(handles):
        return None, None
    return amdsmi, handles[idx]


class GpuTelemetry:
    """Background sampler of one GPU's SMU metrics between ``start()`` and ``stop()``."""

    KEYS_SCLK = ("current_gfxclks", "current_gfxclk", "average_gfxclk_frequency")
    KEYS_MCLK = ("current_uclk", "average_uclk_frequency")
    ACC = ("ppt_residency_acc", "socket_thm_residency_acc", "prochot_residency_acc", "hbm_thm_residency_acc",
           "vr_thm_residency_acc")

    def __init__(self, local_rank: int = 0, interval: float = 0.25):
        self.interval = interval
        self.smi, self.h = _amdsmi_handle(local_rank)
        self.samples: List[Dict[str, Any]] = []
        self._stop = threading.Event()
        self._thr: Optional[threading.Thread] = None
        self._m0: Optional[Dict[str, Any]] = None
        self._m1: Optional[Dict[str, Any]] = None

    @property
    def available(self) -> bool:
        return self.h is not None

    def _metrics(self) -> Optional[Dict[str, Any]]:
        try:
            return self.smi.amdsmi_get_gpu_metrics_info(self.h)
        except Exception:
            return None

    def _first(self, m, keys):
        for k in keys:
            v = _num(m.get(k))
            if v is not None:
                return v
        return None

    def _loop(self):
        while not self._stop.is_set():
            m = self._metrics()
            if m is not None:
                self.samples.append({
                    "sclk": self._first(m, self.KEYS_SCLK), "mclk": self._first(m, self.KEYS_MCLK),
                    "power": self._first(m, ("current_socket_power", "average_socket_power")),
                    "hotspot": _num(m.get("temperature_hotspot")), "hbm": _num(m.get("temperature_mem")),
                    "throttle": m.get("throttle_status"), "indep": m.get("indep_throttle_status")})
            self._stop.wait(self.interval)

    def start(self) -> "GpuTelemetry":
        if not self.available:
            return self
        self._m0 = self._metrics()
        self._thr = threading.Thread(target=self._loop, name="bllm-telemetry", daemon=True)
        self._thr.start()
        return self

    def stop(self) -> Dict[str, Any]:
        if self._thr is not None:
            self._stop.set()
            self._thr.join(timeout=5)
        self._m1 = self._metrics() if self.available else None
        return self.summary()

    def summary(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {"source": "amdsmi gpu_metrics" if self.available else None,
                               "samples": len(self.samples)}
        names = ("sclk_mhz", "mclk_mhz", "power_w", "hotspot_c", "hbm_c")
        for key, name in zip(("sclk", "mclk", "power", "hotspot", "hbm"), names):
            vals = [s[key] for s in self.samples if s[key] is not None]
            if name in ("sclk_mhz", "mclk_mhz", "power_w"):
                out[name + "_avg"] = round(sum(vals) / len(vals), 1) if vals else None
            if name in ("sclk_mhz",):
                out[name + "_min"] = round(min(vals), 1) if vals else None
            if name in ("power_w", "hotspot_c", "hbm_c"):
                out[name + "_max"] = round(max(vals), 1) if vals else None
        thr = [s["throttle"] for s in self.samples if isinstance(s["throttle"], int) and s["throttle"] not in _NA]
        out["throttle_status_nonzero_frac"] = round(sum(1 for t in thr if t) / len(thr), 3) if thr else None
        # residency accumulators: fraction of the region spent under each limit
        res = None
        m0, m1 = self._m0, self._m1
        if m0 and m1:
            c0, c1 = _num(m0.get("accumulation_counter")), _num(m1.get("accumulation_counter"))
            if c0 is not None and c1 is not None and c1 > c0:
                res = {}
                for k in self.ACC:
                    a0, a1 = _num(m0.get(k)), _num(m1.get(k))
                    if a0 is not None and a1 is not None:
                        res[k.replace("_residency_acc", "")] = round((a1 - a0) / (c1 - c0), 4)
            xg = {}
            for k in ("xgmi_read_data_acc", "xgmi_write_data_acc"):
                a0, a1 = m0.get(k), m1.get(k)
                if isinstance(a0, (list, tuple)) and isinstance(a1, (list, tuple)):
                    d = [b - a for a, b in zip(a0, a1) if a not in _NA and b not in _NA and b >= a]
                    xg[k.replace("_data_acc", "_kb")] = sum(d) if d else None
            if xg:
                out["xgmi"] = xg
        out["limit_residency"] = res
        return out


def library_versions() -> Dict[str, Any]:
    """torch / HIP / ROCm / hipBLASLt / rocBLAS versions (the TunableOp validators' keys)."""
    out: Dict[str, Any] = {}
    try:
        import torch
        out["torch"] = torch.__version__
        out["hip"] = torch.version.hip
        if torch.cuda.is_available():
            v = dict(torch.cuda.tunable.get_validators())
            out["hipblaslt"] = v.get("HIPBLASLT_VERSION")
            out["rocblas"] = v.get("ROCBLAS_VERSION")
            out["gcn_arch"] = v.get("GCN_ARCH_NAME")
    except Exception:
        pass
    try:
        with open("/opt/rocm/.info/version") as f:
            out["rocm"] = f.read().strip()
    except Exception:
        out["rocm"] = None
    return out


def tunableop_status(path: Optional[str]) -> Optional[Dict[str, Any]]:
    """Was the TunableOp results file accepted?  Compares its Validator lines with this process's
    validators (a mismatch makes TunableOp ignore the file and keep hipBLASLt's heuristic) and
    counts the file's result rows against the results TunableOp holds after the run."""
    if not path:
        return None
    out: Dict[str, Any] = {"file": os.path.basename(path)}
    rows, file_val = 0, {}
    try:
        with open(path) as f:
            for line in f:
                parts = line.strip().split(",")
                if len(parts) >= 3 and parts[0] == "Validator":
                    file_val[parts[1]] = ",".join(parts[2:])
                elif len(parts) >= 4:
                    rows += 1
    except OSError:
        out["error"] = "unreadable"
        return out
    out["file_rows"] = rows
    try:
        import torch
        live = dict(torch.cuda.tunable.get_validators())
        mism = {k: {"file": v, "live": live.get(k)} for k, v in file_val.items() if live.get(k) != v}
        out["validators_match"] = not mism
        out["mismatch"] = mism or None
        res = torch.cuda.tunable.get_results()
        out["results_held"] = len(res)
        out["enabled"] = bool(torch.cuda.tunable.is_enabled())
    except Exception as e:   # CPU box / API drift
        out["validators_match"] = None
        out["error"] = type(e).__name__
    return out


def rccl_debug_env(rank: int, directory: Optional[str] = None) -> Optional[str]:
    """Ask RCCL to log its init-time topology decisions (``NCCL_DEBUG=INFO``, subsystems INIT and
    GRAPH only: no per-collective lines) to a per-rank file; returns the path.  Must run before
    the process group is created.  A user's own ``NCCL_DEBUG_FILE`` is kept (and parsed); a
    preset ``NCCL_DEBUG`` level (images often set WARN / VERSION) is raised to INFO into the file,
    so RCCL's warnings land there too."""
    import os
    import tempfile
    if os.environ.get("NCCL_DEBUG_FILE"):
        os.environ.setdefault("NCCL_DEBUG", "INFO")
        return os.environ["NCCL_DEBUG_FILE"]
    path = os.path.join(directory or tempfile.gettempdir(), f"bllm_rccl_{os.getuid()}_{os.getpid()}_r{rank}.log")
    os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,GRAPH", NCCL_DEBUG_FILE=path)
    return path


def rccl_topology(path: Optional[str], max_lines: int = 24) -> Optional[Dict[str, Any]]:
    """What RCCL chose at init, from its INIT/GRAPH log: ranks / nodes, the channel counts per
    kind, the ring and tree orders of the first channels, and the algorithm/protocol threshold
    lines (the per-collective choice RCCL's tuner makes from them)."""
    import os
    import re
    if not path or not os.path.exists(path):
        return None
    lines = [ln.rstrip() for ln in open(path, errors="replace") if "NCCL INFO" in ln]
    out: Dict[str, Any] = {"log": path, "lines": len(lines)}
    keep = []
    for ln in lines:
        msg = ln.split("NCCL INFO", 1)[1].strip()
        m = re.search(r"nRanks (\d+) nNodes (\d+) localRanks (\d+)", msg)
        if m:
            out.update(n_ranks=int(m.group(1)), n_nodes=int(m.group(2)), local_ranks=int(m.group(3)))
        m = re.search(r"(\d+) coll channels, (?:(\d+) collnet channels, )?(?:(\d+) nvls channels, )?(\d+) p2p channels", msg)
        if m:
            out.update(coll_channels=int(m.group(1)), p2p_channels=int(m.group(4)))
        if re.match(r"Channel \d+/\d+ :", msg):
            out["channels"] = max(out.get("channels", 0), int(msg.split()[1].split("/")[1]))
            if len(out.setdefault("rings", [])) < 4:
                out["rings"].append(msg)
        elif re.match(r"Tree \d+ :", msg):
            out["trees"] = out.get("trees", 0) + 1
            if len(out.setdefault("tree_examples", [])) < 2:
                out["tree_examples"].append(msg)
        elif re.search(r"Trees|threadThresholds|Algo|algorithm|Protocol|Usable|Connected all|NET/|P2P|xGMI|XGMI",
                       msg) and len(keep) < max_lines:
            keep.append(msg)
    out["decisions"] = keep
    return out
