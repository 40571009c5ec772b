"""GPU clock / power trace around the headline bench (round-2 verdict item 7).

A side thread samples amd-smi's GPU metrics (gfx clock, socket power, temperature, throttle status)
every ~2 ms while this process runs bench.py in-process; prints one JSON object: the samples
(seconds from the bench start) and the bench's own JSON line.

    python tools/probes/clock_trace.py [bench.py args ...]
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.append("/opt/rocm/share/amd_smi")

KEYS = ("gfxclk", "power", "temperature_hotspot", "throttle", "gfx_activity", "uclk")


def sampler(stop, out, t0):
    try:
        import amdsmi

        amdsmi.amdsmi_init()
        h = amdsmi.amdsmi_get_processor_handles()[0]
    except Exception as e:  # no amd-smi access on this box
        out.append({"error": f"amdsmi: {e}"})
        return
    while not stop.is_set():
        t = time.perf_counter() - t0
        try:
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            s = {"t": round(t, 4)}
            for k, v in m.items():
                if any(x in k for x in KEYS) and not isinstance(v, (list, dict)):
                    s[k] = v
            out.append(s)
        except Exception as e:
            out.append({"t": round(t, 4), "error": str(e)})
            return
        time.sleep(0.002)


def main():
    import bench

    samples = []
    stop = threading.Event()
    t0 = time.perf_counter()
    th = threading.Thread(target=sampler, args=(stop, samples, t0), daemon=True)
    th.start()
    time.sleep(0.2)  # idle baseline
    buf = io.StringIO()
    t_bench = time.perf_counter() - t0
    with contextlib.redirect_stdout(buf):
        rc = bench.main(sys.argv[1:])
    t_end = time.perf_counter() - t0
    time.sleep(0.2)
    stop.set()
    th.join()
    line = next((ln for ln in reversed(buf.getvalue().splitlines()) if ln.startswith("{")), None)
    print(json.dumps({"rc": rc, "bench_start_s": t_bench, "bench_end_s": t_end, "bench": json.loads(line) if line else None,
                      "samples": samples}))


if __name__ == "__main__":
    main()
