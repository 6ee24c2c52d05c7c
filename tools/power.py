"""Board power and GFX clock of one GPU, sampled while a bench region runs (measurement only).

    with PowerSampler("0000:05:00.0") as ps:
        ... timed launches ...
    ps.summary() -> {"samples": n, "mean_W": .., "max_W": .., "clock_MHz_mean": .., ...}

Reads amdsmi (the ROCm SMI library's Python binding) in a background thread every `period`
seconds: current socket power (W) and the GFX clock (MHz) of the device whose PCI address
matches.  No HIP call, so it neither initialises nor touches the HIP context.  Every failure
(no amdsmi, no permission, device not found) turns into {"error": ...}: a reported sample,
never a reason to lose the bench line.
"""
from __future__ import annotations

import threading
import time


def _handle(bdf: str):
    import amdsmi
    amdsmi.amdsmi_init()
    for h in amdsmi.amdsmi_get_processor_handles():
        if amdsmi.amdsmi_get_gpu_device_bdf(h).lower() == bdf.lower():
            return amdsmi, h
    raise LookupError(f"amdsmi lists no GPU at {bdf}")


class PowerSampler:
    def __init__(self, bdf: str, period: float = 0.05):
        self.bdf, self.period = bdf, period
        self.samples: list[tuple[float, float, float]] = []  # (t, W, MHz)
        self.error = None
        self._stop = threading.Event()
        self._thread = None
        self.limit_W = None

    def _run(self, smi, h):
        clk = smi.AmdSmiClkType.GFX
        while not self._stop.is_set():
            try:
                p = smi.amdsmi_get_power_info(h)
                w = p.get("current_socket_power")
                if not isinstance(w, (int, float)) or w in (0, "N/A"):
                    w = p.get("average_socket_power")
                c = smi.amdsmi_get_clock_info(h, clk).get("clk")
                self.samples.append((time.perf_counter(), float(w), float(c)))
            except Exception as e:  # noqa: BLE001 -- reported in the summary
                self.error = f"{type(e).__name__}: {e}"
                return
            self._stop.wait(self.period)

    def __enter__(self):
        try:
            smi, h = _handle(self.bdf)
            try:
                self.limit_W = smi.amdsmi_get_power_info(h).get("power_limit")
            except Exception:  # noqa: BLE001
                pass
            self._thread = threading.Thread(target=self._run, args=(smi, h), daemon=True)
            self._thread.start()
        except Exception as e:  # noqa: BLE001
            self.error = f"{type(e).__name__}: {e}"
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2)
        return False

    def summary(self) -> dict:
        if not self.samples:
            return {"error": self.error or "no samples"}
        w = [s[1] for s in self.samples]
        c = [s[2] for s in self.samples]
        # the busy part of the region: samples whose clock is above half the region's peak
        # (the first samples can precede the kernels' ramp-up)
        busy = [s for s in self.samples if s[2] > 0.5 * max(c)] or self.samples
        res = {"source": "amdsmi current_socket_power / GFX clk, "
                         f"every {self.period * 1e3:.0f} ms during the timed launches",
               "samples": len(w), "mean_W": round(sum(w) / len(w), 1), "max_W": round(max(w), 1),
               "busy_mean_W": round(sum(s[1] for s in busy) / len(busy), 1),
               "clock_MHz_mean": round(sum(c) / len(c), 1),
               "busy_clock_MHz_mean": round(sum(s[2] for s in busy) / len(busy), 1)}
        if self.limit_W is not None:
            res["power_limit"] = self.limit_W
        if self.error:
            res["error"] = self.error
        return res
