"""Config 5 host -> host (214 numpy gradients) through _reduce_grads at one rank, a few calls: the
program tools/gpu_host_copy_trace.sh runs under rocprofv3 --memory-copy-trace to see each piece's
H2D and D2H on the DMA engines."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    import tips_amd
    torch.cuda.set_device(0)
    tips_amd.init()
    sizes = bench.resnet50_grad_sizes()
    hg = [np.random.default_rng(i).random(k, dtype=np.float32) for i, k in enumerate(sizes)]
    for _ in range(3):
        outs = tips_amd._reduce_grads(hg)
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
        t0 = time.perf_counter()
        outs = tips_amd._reduce_grads(hg)
        print("call ms %.3f" % ((time.perf_counter() - t0) * 1e3), flush=True)
    assert all(np.array_equal(o, g) for o, g in zip(outs, hg))


if __name__ == "__main__":
    main()
