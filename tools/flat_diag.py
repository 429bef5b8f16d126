"""flat_diag.py — tests/test_gpu_allreduce.py::test_fused_flat_outputs' failing case, with a report of
what differs (which tensors, where, how many elements), under the current TIPS_FUSION_CALLER_STREAM.

usage: python3 tools/flat_diag.py [threshold] [measure_pack]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    thr = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    mp = sys.argv[2] if len(sys.argv) > 2 else "0"
    os.environ["TIPS_FUSION_THRESHOLD"] = str(thr)
    os.environ["TIPS_FUSION_MEASURE_PACK"] = mp
    import torch
    import tips_amd
    tips_amd.init()
    tdt = [torch.float32, torch.float64, torch.int32, torch.int64, torch.float16, torch.bfloat16]
    rng = np.random.default_rng(thr % 1000 + int(mp))
    bad = 0
    for dt in tdt:
        sizes = [int(round(2 ** rng.uniform(0, 15))) for _ in range(120)] + [0, 3, 1, 40000, 7]
        base = torch.randint(-1000, 1000, (sum(sizes) + len(sizes) + 2,), device="cuda").to(dt)
        ins, off = [], 1
        for s in sizes:
            ins.append(base[off:off + s])
            off += s + 1
        for it in range(2):
            outs = tips_amd.fused_allreduce_flat(ins)
            torch.cuda.synchronize()
            for i, (o, t) in enumerate(zip(outs, ins)):
                if not torch.equal(o, t):
                    d = (o != t).nonzero().flatten()
                    bad += 1
                    print("dtype %s call %d tensor %d (n %d, in ptr %% 16 = %d, out ptr %% 16 = %d): %d differ, first %d "
                          "last %d; got %s want %s" % (dt, it, i, t.numel(), t.data_ptr() % 16, o.data_ptr() % 16,
                                                        d.numel(), d[0].item(), d[-1].item(), o[d[:4]].tolist(),
                                                        t[d[:4]].tolist()), flush=True)
            del outs
    print("caller_stream=%s threshold %d measure %s: %d bad" % (os.environ.get("TIPS_FUSION_CALLER_STREAM", "1"), thr,
                                                                 mp, bad), flush=True)


if __name__ == "__main__":
    main()
