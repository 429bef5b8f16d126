"""One shape of the direct schedule's fold for PMC passes (tools/gpu_pmc_multi.sh): 8 sources of one
32 MiB sub-chunk (config 3's direct shape at K = 4) folded into a destination, over 4 rotating
buffer sets (HBM-only operands), 24 launches. Algorithmic bytes per launch: 9 x 32 MiB."""
import sys

import torch

sys.path.insert(0, ".")
from tips_amd import _lib  # noqa: E402

torch.cuda.set_device(0)
s = torch.cuda.current_stream()
p, n = 8, 32 << 18
sets = []
for k in range(4):
    srcs = [torch.randn(n, device="cuda") for _ in range(p)]
    dst = torch.empty(n, device="cuda")
    ptrs, keep = _lib.ptr_array([t.data_ptr() for t in srcs])
    sets.append((srcs, dst, ptrs, keep))
for i in range(24):
    srcs, dst, ptrs, _ = sets[i % 4]
    _lib.call("tips_multi_sum", dst.data_ptr(), ptrs, p, n, _lib.FLOAT32, s.cuda_stream)
torch.cuda.synchronize()
srcs, dst, _, _ = sets[23 % 4]
ref = srcs[0].clone()
for t in srcs[1:]:
    ref += t
print("fold bit-exact vs torch rank-order sum:", bool(torch.equal(dst, ref)))
