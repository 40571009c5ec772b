"""Does data read at the end of one pass survive in the MI355X Infinity Cache (MALL, 256 MB) for the
start of the next?  Times a torch sum over a chunk of B MB read right after itself (warm) vs right
after 4 GB of other reads (cold), for several chunk sizes; prints one JSON line."""
import json

import torch


def t(fn, reps=20):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    out = []
    for a, b in ev:
        fn[0]()
        a.record()
        fn[1]()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) * 1e3 for a, b in ev)[reps // 2]


def main():
    big = torch.ones(4 << 30 >> 3, dtype=torch.float64, device="cuda")  # 4 GB of other data
    res = {}
    for mb in (32, 64, 128, 192, 256, 384, 512):
        x = torch.ones((mb << 20) >> 3, dtype=torch.float64, device="cuda")
        warm = t((lambda: x.sum(), lambda: x.sum()))
        cold = t((lambda: big.sum(), lambda: x.sum()))
        res[mb] = {"warm_us": round(warm, 1), "cold_us": round(cold, 1),
                   "warm_TBps": round(mb * 2**20 / warm / 1e6, 2), "cold_TBps": round(mb * 2**20 / cold / 1e6, 2)}
        del x
    print(json.dumps(res))


if __name__ == "__main__":
    main()
