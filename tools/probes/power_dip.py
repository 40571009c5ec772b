"""Is the slow stretch after an idle period (profiles/round2/s2_prof/per_call_grad_us.txt) the platform's
power management or the gradient kernel?  Times back-to-back reads of 8 GB with torch (a plain
sum, no LDS, no replicas) after an idle second, per call, with HIP events.  Prints one JSON line."""
import json
import time

import torch


def main():
    x = torch.ones(1_000_000_000, dtype=torch.float64, device="cuda")  # 8 GB
    out = {}
    for name, fn in (("sum", lambda: x.sum()), ("copy_half", lambda: x[: 500_000_000].clone())):
        fn()
        torch.cuda.synchronize()
        time.sleep(1.0)  # idle, like the bench between setup and the first round
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(40)]
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        out[name] = [round(a.elapsed_time(b) * 1e3, 1) for a, b in ev]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
