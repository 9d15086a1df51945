"""GPU telemetry via amdsmi (replaces the NVML system metrics Aim collected for the reference, O3).

``gpu_stats()`` returns per-device utilisation, VRAM, power and temperature when amdsmi is usable,
else falls back to torch's allocator counters. Never initialises anything on import.
"""
from __future__ import annotations

from typing import Dict, List


def gpu_stats() -> List[Dict[str, float]]:
    out = []
    try:
        import amdsmi  # type: ignore
        amdsmi.amdsmi_init()
        try:
            for i, h in enumerate(amdsmi.amdsmi_get_processor_handles()):
                rec = {"index": i}
                try:
                    act = amdsmi.amdsmi_get_gpu_activity(h)
                    rec["gfx_util"] = float(act.get("gfx_activity", 0))
                    rec["mem_util"] = float(act.get("umc_activity", 0))
                except Exception:
                    pass
                try:
                    vu = amdsmi.amdsmi_get_gpu_vram_usage(h)
                    rec["vram_used_mb"] = float(vu.get("vram_used", 0))
                    rec["vram_total_mb"] = float(vu.get("vram_total", 0))
                except Exception:
                    pass
                try:
                    rec["temp_c"] = float(amdsmi.amdsmi_get_temp_metric(
                        h, amdsmi.AmdSmiTemperatureType.HOTSPOT, amdsmi.AmdSmiTemperatureMetric.CURRENT))
                except Exception:
                    pass
                try:
                    pw = amdsmi.amdsmi_get_power_info(h)
                    rec["power_w"] = float(pw.get("current_socket_power", pw.get("average_socket_power", 0)) or 0)
                except Exception:
                    pass
                out.append(rec)
        finally:
            amdsmi.amdsmi_shut_down()
    except Exception:
        import torch
        if torch.cuda.is_available():
            for i in range(torch.cuda.device_count()):
                out.append({"index": i, "torch_allocated_mb": torch.cuda.memory_allocated(i) / 2**20,
                            "torch_reserved_mb": torch.cuda.memory_reserved(i) / 2**20})
    return out


def memory_report(device=None) -> Dict[str, float]:
    import torch
    if not torch.cuda.is_available():
        return {}
    return {"hbm_allocated_gb": torch.cuda.memory_allocated(device) / 1e9,
            "hbm_reserved_gb": torch.cuda.memory_reserved(device) / 1e9,
            "hbm_peak_gb": torch.cuda.max_memory_allocated(device) / 1e9}


def system_log_entries(stats: List[Dict[str, float]] = None) -> Dict[str, float]:
    """Flatten ``gpu_stats()`` into tracker keys ``sys_gpu{i}_{metric}`` (logged with context subset=system)."""
    stats = gpu_stats() if stats is None else stats
    out = {}
    for rec in stats:
        i = int(rec.get("index", 0))
        for k, v in rec.items():
            if k != "index" and isinstance(v, (int, float)):
                out[f"sys_gpu{i}_{k}"] = float(v)
    return out
