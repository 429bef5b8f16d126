"""CPU: backward-overlapped gradient buckets (tips_amd.optim._GradBuckets).

The reference's per-gradient MPIAllreduce ops start as their gradients appear during backward
(__init__.py:212-222, async op kernel ops.cc:86-115). Here post-accumulate grad hooks issue one
in-place allreduce per bucket of the reversed parameter list. These tests run the hooks on CPU
tensors with a stand-in allreduce (multiply by the number of ranks: every rank's gradient equal),
so the layout, the issue order, the pass counting and the error paths are checked without a GPU.
The same class over real RCCL ranks: tests/test_gpu_rccl_procs.py::test_overlapped_optimizer_over_rccl.
"""
import random

import pytest
import torch

from tips_amd.optim import _GradBuckets

RANKS = 3


def make_model(seed=0, widths=(16, 32, 32, 24, 8)):
    torch.manual_seed(seed)
    layers = []
    for a, b in zip(widths[:-1], widths[1:]):
        layers += [torch.nn.Linear(a, b), torch.nn.Tanh()]
    return torch.nn.Sequential(*layers[:-1])


def loss_of(m, seed=1):
    g = torch.Generator().manual_seed(seed)
    return m(torch.randn(5, m[0].in_features, generator=g)).pow(2).sum()


def local_grads(seed_model=0, seeds=(1,)):
    m = make_model(seed_model)
    for s in seeds:
        loss_of(m, s).backward()
    return [p.grad.clone() for p in m.parameters()]


def padded(p):
    """A parameter's extent in the flat buffer: its elements rounded up to 256 B."""
    al = 256 // p.element_size()
    return (p.numel() + al - 1) // al * al


def buckets_for(m, bucket_bytes, passes=1, average=False):
    calls = []

    def issue(flat):
        calls.append(flat.numel())
        flat.mul_(RANKS)

    gb = _GradBuckets(list(m.parameters()), bucket_bytes, passes, average, issue=issue)
    return gb, calls


def test_layout_reversed_contiguous_and_bounded():
    m = make_model()
    params = list(m.parameters())
    gb, _ = buckets_for(m, bucket_bytes=2048)
    # reverse order: the last parameter sits at offset 0 of the flat buffer
    assert gb.where[id(params[-1])][2] == 0
    prev_end = 0
    for key, s, e, ps in gb.buckets:
        assert s == prev_end and e > s
        prev_end = e
        assert sum(padded(p) for p in ps) == e - s
        assert sum(p.numel() * 4 for p in ps) <= 2048 or len(ps) == 1  # one oversized parameter alone
        for p in ps:
            b, k, off = gb.where[id(p)]
            assert s <= off and off + p.numel() <= e and off * 4 % 256 == 0  # 256-B aligned slices
    assert prev_end == sum(padded(p) for p in params)
    assert [p for b in gb.buckets for p in b[3]] == params[::-1]
    gb.remove()


def test_buckets_issue_in_index_order_whatever_the_hook_order():
    m = make_model()
    gb, _ = buckets_for(m, bucket_bytes=1024)
    for p in m.parameters():
        p.grad = torch.ones_like(p)
    ps = list(m.parameters())
    random.Random(7).shuffle(ps)
    for p in ps:
        gb._hook(p, final_pass=True, active=True)
        issued = [t for t in gb.issue_log]
        assert issued == list(range(len(issued)))  # always a prefix of 0, 1, 2, ...
    assert gb.issue_log == list(range(len(gb.buckets)))
    gb.synchronize()
    assert gb.last_issue_log == list(range(len(gb.buckets)))
    for p in m.parameters():
        assert torch.equal(p.grad, torch.full_like(p, RANKS))
    gb.remove()


def test_real_backward_issues_during_backward_and_sums():
    exp = [g * RANKS for g in local_grads()]
    m = make_model()
    gb, calls = buckets_for(m, bucket_bytes=1536)
    loss_of(m).backward()
    # every bucket was complete by the end of backward, so every one was issued by the hooks
    assert gb.issue_log == list(range(len(gb.buckets))) and len(gb.buckets) > 2
    gb.synchronize()
    for p, e in zip(m.parameters(), exp):
        assert torch.equal(p.grad, e)
        assert p.grad.data_ptr() == gb.view(p).data_ptr()  # .grad is the bucket view
    # a second iteration with set_to_none=False accumulates straight into the views
    for p in m.parameters():
        p.grad.zero_()
    loss_of(m).backward()
    gb.synchronize()
    for p, e in zip(m.parameters(), exp):
        assert torch.equal(p.grad, e)
    assert sum(calls) == 2 * sum(padded(p) for p in m.parameters())
    gb.remove()


def test_accumulation_passes_and_average():
    acc = local_grads(seeds=(1, 2))  # torch accumulates two backwards into .grad
    m = make_model()
    gb, _ = buckets_for(m, bucket_bytes=1536, passes=2, average=True)
    state = {"pass": 0}
    gb.final_pass = lambda: state["pass"] == 1
    loss_of(m, 1).backward()
    assert gb.issue_log == []  # the first pass only accumulates into the views
    state["pass"] = 1
    loss_of(m, 2).backward()
    assert gb.issue_log == list(range(len(gb.buckets)))
    gb.synchronize()
    for p, a in zip(m.parameters(), acc):
        assert torch.equal(p.grad, (a / 2) * RANKS)
    gb.remove()


def test_unused_parameter_contributes_zeros_and_stays_none():
    m = make_model()
    extra = torch.nn.Parameter(torch.randn(7))
    gb = _GradBuckets(list(m.parameters()) + [extra], 1 << 20, 1, False, issue=lambda f: f.mul_(RANKS))
    loss_of(m).backward()
    # extra sits in bucket 0 (reversed order) and never gets a gradient: nothing issued by the hooks
    assert gb.issue_log == []
    gb.synchronize()
    assert extra.grad is None
    assert torch.equal(gb.view(extra), torch.zeros(7))
    exp = [g * RANKS for g in local_grads()]
    for p, e in zip(m.parameters(), exp):
        assert torch.equal(p.grad, e)
    gb.remove()


def test_synchronize_without_backward_issues_bucket_by_bucket_unless_told():
    """How far the hooks got is rank-local, so synchronize() always issues the rest bucket by
    bucket; one allreduce per group only on the caller's word that no backward ran anywhere."""
    m = make_model()
    gb, calls = buckets_for(m, bucket_bytes=512)
    for p in m.parameters():
        p.grad = torch.full_like(p, 2.0)
    gb.synchronize()
    assert gb.last_issue_log == list(range(len(gb.buckets))) and len(calls) == len(gb.buckets) > 1
    for p in m.parameters():
        assert torch.equal(p.grad, torch.full_like(p, 2.0 * RANKS))
    calls.clear()
    gb.synchronize(whole_groups=True)
    assert len(calls) == 1 and calls[0] == sum(padded(p) for p in m.parameters())
    assert gb.last_issue_log == [("group", (torch.float32, torch.device("cpu")))]
    for p in m.parameters():
        assert torch.equal(p.grad, torch.full_like(p, 2.0 * RANKS ** 2))
    loss_of(m).backward()  # the hooks issue buckets: whole_groups would not pair across ranks
    with pytest.raises(RuntimeError, match="would not pair"):
        gb.synchronize(whole_groups=True)
    gb.remove()


def test_second_backward_after_issue_is_an_error():
    m = make_model()
    gb, _ = buckets_for(m, bucket_bytes=1536)
    loss_of(m).backward()
    loss_of(m).backward()
    with pytest.raises(RuntimeError, match="accumulated again"):
        gb.synchronize()
    gb.remove()


def test_mixed_dtypes_make_separate_groups():
    m = make_model()
    m[-1].double()
    gb, calls = buckets_for(m, bucket_bytes=1 << 20)
    keys = [b[0] for b in gb.buckets]
    assert keys[0][0] == torch.float64 and all(k[0] == torch.float32 for k in keys[1:])
    loss = m[-1](m[:-1](torch.randn(3, 16)).double()).pow(2).sum()
    loss.backward()
    gb.synchronize()
    assert gb.last_issue_log == [0, 1]
    gb.remove()


def test_newest_owner_reduces_and_dropped_owner_is_collected():
    import gc
    import weakref
    m = make_model()
    old, old_calls = buckets_for(m, bucket_bytes=1536)
    new, new_calls = buckets_for(m, bucket_bytes=1536)  # wrapping the same parameters again
    loss_of(m).backward()
    assert old.issue_log == [] and new.issue_log == list(range(len(new.buckets)))
    new.synchronize()
    exp = [g * RANKS for g in local_grads()]
    for p, e in zip(m.parameters(), exp):
        assert torch.equal(p.grad, e)  # reduced once, not twice
    ref = weakref.ref(new)
    del new, old
    gc.collect()
    assert ref() is None  # the hooks do not keep the buckets alive
    for p in m.parameters():
        p.grad = None
    loss_of(m).backward()  # hooks of a collected owner do nothing
    assert torch.equal(list(m.parameters())[0].grad, local_grads()[0])


def _gloo_worker(rank, world, port, q):
    import os
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import datetime
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    from tips_amd.optim import _GradBuckets
    try:
        m = make_model()
        gb = _GradBuckets(list(m.parameters()), 1024, 1, False, issue=lambda f: dist.all_reduce(f))
        # every rank's hooks fire in its own order: the allreduces must still pair bucket for bucket
        for p in m.parameters():
            p.grad = torch.full_like(p, float(rank + 1))
        ps = list(m.parameters())
        random.Random(100 + rank).shuffle(ps)
        for p in ps:
            gb._hook(p, final_pass=True, active=True)
        gb.synchronize()
        tot = world * (world + 1) / 2
        ok1 = all(torch.equal(p.grad, torch.full_like(p, tot)) for p in m.parameters())
        # a real backward with rank-specific batches: sums equal the sum of every rank's gradients
        for p in m.parameters():
            p.grad.zero_()
        loss_of(m, seed=10 + rank).backward()
        gb.synchronize()
        exp = None
        for r in range(world):
            g = local_grads(seeds=(10 + r,))
            exp = g if exp is None else [a + b for a, b in zip(exp, g)]
        ok2 = all(torch.allclose(p.grad, e, rtol=1e-6, atol=1e-6) for p, e in zip(m.parameters(), exp))
        # a parameter that gets a gradient on some ranks only, in the FIRST bucket (the last
        # parameter): on rank 0 the hooks issue nothing during backward, elsewhere every bucket.
        # The allreduces still pair (a whole-group allreduce on rank 0 would not: gloo raises on
        # the size mismatch, or the ranks hang until the timeout).
        m3 = make_model()
        extra = torch.nn.Parameter(torch.full((7,), 1.0))
        ps3 = list(m3.parameters()) + [extra]
        gb3 = _GradBuckets(ps3, 1024, 1, False, issue=lambda f: dist.all_reduce(f))
        out = m3(torch.randn(5, 16, generator=torch.Generator().manual_seed(30 + rank))).pow(2).sum()
        if rank != 0:
            out = out + (extra * float(rank)).sum()
        out.backward()
        hooks_issued = list(gb3.issue_log)
        gb3.synchronize()
        ok3 = torch.equal(gb3.view(extra), torch.full((7,), float(sum(range(world)))))
        ok3 = ok3 and (extra.grad is None) == (rank == 0)
        ok3 = ok3 and (hooks_issued == []) == (rank == 0) and gb3.last_issue_log == list(range(len(gb3.buckets)))
        q.put((rank, ok1, ok2 and ok3, len(gb.buckets)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bucket_order_pairs_across_gloo_ranks(world):
    """World-size 2 / 3 gloo groups, torch.distributed.all_reduce standing in for tips_allreduce:
    hooks fired in a different order on every rank still issue the same allreduces in the same
    order (a mismatch would pair buckets of different sizes: an error or a hang)."""
    import socket
    import torch.multiprocessing as tmp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, ok1, ok2, nb in res:
        assert ok1 and ok2 and nb > 3, (rank, ok1, ok2, nb)


def test_end_of_backward_callback_joins_once_per_backward():
    """A backward that issued buckets queues one autograd final callback, which orders the
    streams the buckets were issued from after the side streams (on CPU: counted only)."""
    m = make_model()
    gb, _ = buckets_for(m, bucket_bytes=1536)
    loss_of(m).backward()
    assert getattr(gb, "backward_joins", 0) == 1 and not gb._cb_queued
    gb.synchronize()
    for p in m.parameters():
        p.grad.zero_()
    loss_of(m).backward()
    assert gb.backward_joins == 2
    gb.synchronize()
    gb.remove()
