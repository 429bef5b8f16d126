"""DistributedOptimizer and DistributedGradientTape for torch — mirror
tips.tensorflow.DistributedOptimizer / DistributedGradientTape
(reference tips/tensorflow/__init__.py:252-456, 460-569).

The reference wraps a TF optimizer: compute_gradients() allreduces every
gradient (_make_allreduce_grads_fn, __init__.py:189-227) before the wrapped
optimizer applies them, optionally after backward_passes_per_step local
accumulations (LocalGradientAggregationHelper, gradient_aggregation.py). Here
the wrapped object is a torch.optim.Optimizer: the parameters' .grad tensors
are summed over ranks in place and then the wrapped optimizer steps. Dense
device gradients are views of per-dtype flat buffers cut into <= 25 MiB buckets,
allreduced in place either during backward as each bucket completes
(_GradBuckets, as the reference's async per-gradient ops overlap backward) or
after it, in step(). Which one is measured, not assumed (TIPS_OVERLAP_BACKWARD=
auto, the default): the first optimizer steps alternate the two, every rank
times them on the device, the ranks agree on the slowest rank's means and all
keep the faster (_OverlapChoice). Round 3's default was "during"; rehearsals on
one shared GPU measured it both faster and slower. =1 / =0 fix
the choice. The rest go through tips_amd.allreduce_grads.

As in the reference, op / prescale / postscale never reach the reduction
(__init__.py:82-87, 194-201): the gradients are SUMMED over ranks, op=Average
included. gradient_predivide_factor is validated as the
reference validates it (__init__.py:408-411) and otherwise has no effect,
for the same reason.
"""
import warnings

Average = 'Average'


def _allreduce_flat_(flat):
    """In-place SUM of one contiguous device tensor over the ranks (tips_allreduce, in == out)."""
    from . import _lib, basics, tensors
    basics.init()
    _lib.call("tips_allreduce", flat.data_ptr(), flat.data_ptr(), flat.numel(), tensors.dtype_code(flat), _lib.OP_SUM,
              tensors.stream_of(flat))


def _remove_hooks(handles):
    for h in handles:
        h.remove()


class _GradBuckets(object):
    """Gradient buckets whose allreduces start during backward.

    In the reference every gradient's MPIAllreduce is an async op of the TF graph
    (__init__.py:212-222, ops.cc:86-115): it starts as soon as its gradient exists, while the
    rest of backward still runs. The torch mirror gets the same overlap from post-accumulate
    grad hooks. The parameters are laid out in REVERSE order (backward produces the last layer's
    gradients first) in one flat buffer per (dtype, device), and cut into buckets of at most
    `bucket_bytes`; every .grad becomes a view of its slice. When the last gradient of a bucket
    has been accumulated, the bucket's slice is allreduced in place on a side stream that waited
    for the backward stream, so the exchange runs beside the remaining backward kernels.

    Ranks must issue the same allreduces in the same order. Buckets are therefore issued strictly
    in index order (a bucket whose gradients are ready waits for every earlier bucket), and the
    layout depends only on the parameter list. synchronize() issues whatever backward did not,
    bucket by bucket in index order (parameters without a gradient contribute zeros), then makes
    the caller's stream wait for the side streams. How far the hooks got is rank-local (a parameter
    may get no gradient on one rank only), so the bucket-by-bucket sequence is what keeps every
    rank's allreduces paired. Only a caller that knows no backward ran on any rank (bench.py's
    optimizer leg) may ask for whole_groups=True: one allreduce of each group's flat buffer.
    `issue(flat_slice)` is the in-place allreduce (a test may pass its own)."""

    def __init__(self, params, bucket_bytes, passes, average, issue=None):
        import threading
        import torch
        self._torch = torch
        self._passes, self._average = int(passes), bool(average)
        self._issue_fn = issue or _allreduce_flat_
        self._lock = threading.Lock()
        self.params = list(params)
        self.groups = {}   # (dtype, device) -> {"n": elements, "flat": tensor}
        self.buckets = []  # [group key, start, end (elements of the group's flat buffer), [params]]
        self.where = {}    # id(param) -> (bucket index, group key, offset)
        cur, cur_bytes = None, 0
        for p in reversed(self.params):
            key = (p.dtype, p.device)
            g = self.groups.setdefault(key, {"n": 0, "flat": None})
            nbytes = p.numel() * p.element_size()
            if cur is None or cur[0] != key or (cur_bytes and cur_bytes + nbytes > bucket_bytes):
                cur = [key, g["n"], g["n"], []]
                self.buckets.append(cur)
                cur_bytes = 0
            self.where[id(p)] = (len(self.buckets) - 1, key, g["n"])
            # every parameter (so every bucket) starts 256-B aligned, as fusion buckets pack
            # (fusion.cc): the kernels' 16-B vector path; the padding stays zero
            al = max(1, 256 // p.element_size())
            g["n"] += (p.numel() + al - 1) // al * al
            cur[2] = g["n"]
            cur[3].append(p)
            cur_bytes += nbytes
        for (dt, dev), g in self.groups.items():
            g["flat"] = torch.zeros(g["n"], dtype=dt, device=dev)
        self._streams = {}
        self.issue_log = []  # (bucket index, or ("group", key)) in issue order, this iteration
        self._reset()
        # The hooks hold this object weakly (a dropped optimizer stops reducing and is collected),
        # and a parameter belongs to the most recent _GradBuckets built over it: wrapping the same
        # parameters again (a new DistributedOptimizer) must not reduce their gradients twice.
        import weakref
        ref = weakref.ref(self)

        def hook(p, _ref=ref):
            gb = _ref()
            if gb is not None and getattr(p, "_tips_grad_buckets", None) is _ref:
                gb._hook(p)

        for p in self.params:
            p._tips_grad_buckets = ref
        self._handles = [p.register_post_accumulate_grad_hook(hook) for p in self.params]
        weakref.finalize(self, _remove_hooks, list(self._handles))

    def remove(self):
        _remove_hooks(self._handles)
        self._handles = []

    def _reset(self):
        self._cb_queued = False
        self._origins = {}  # device -> {stream handle: stream} the buckets were issued from
        self.ready = [0] * len(self.buckets)
        self.issued = [False] * len(self.buckets)
        self.next = 0
        self.seen = set()
        self.sparse = set()  # ids of parameters whose gradient came sparse: reduced by allreduce_grads
        self.error = None

    def view(self, p):
        _, key, off = self.where[id(p)]
        return self.groups[key]["flat"][off:off + p.numel()].view(p.shape)

    def _side(self, device):
        if device.type != "cuda":
            return None
        s = self._streams.get(device)
        if s is None:
            s = self._streams[device] = self._torch.cuda.Stream(device=device)
        return s

    def _adopt(self, p):
        """Make p.grad the view of its slice (copying a gradient autograd allocated elsewhere in);
        a sparse gradient is left alone and its slice zeroed."""
        g, v = p.grad, self.view(p)
        if g is None or g.is_sparse or g.dtype != p.dtype:
            if g is not None:
                self.sparse.add(id(p))
            v.zero_()
            return
        if g.data_ptr() != v.data_ptr():
            v.copy_(g)
            p.grad = v

    def _hook(self, p, final_pass=None, active=None):
        """Post-accumulate grad hook (autograd's device thread, on the backward stream)."""
        if not (self.active() if active is None else active):
            return
        self._adopt(p)
        if not (self.final_pass() if final_pass is None else final_pass):
            return  # an earlier backward of backward_passes_per_step: accumulate into the views only
        with self._lock:
            if id(p) in self.seen:
                self.error = ("a gradient was accumulated again after its bucket's allreduce was issued: "
                              "run one backward per step() (backward_passes_per_step for more)")
                return
            self.seen.add(id(p))
            b = self.where[id(p)][0]
            self.ready[b] += 1
            while self.next < len(self.buckets) and self.ready[self.next] == len(self.buckets[self.next][3]):
                self._issue(self.next)
                self.next += 1
                if not self._cb_queued:
                    # at the end of this backward the streams it ran on wait for the issued
                    # allreduces: whatever the caller does with .grad next (clipping, a norm, step)
                    # is ordered after them, as the reference's compute_gradients hands back reduced
                    # gradients (__init__.py:296-310)
                    try:
                        self._torch.autograd.Variable._execution_engine.queue_callback(self._after_backward)
                        self._cb_queued = True
                    except RuntimeError:  # not inside a backward pass (a direct _hook call)
                        pass

    # the optimizer sets these two
    def active(self):
        return True

    def final_pass(self):
        return True

    def _after_backward(self):
        """Autograd's final callback of a backward that issued buckets: its streams wait for the
        side streams (stream order only; the host does not block)."""
        with self._lock:
            self._cb_queued = False
            for dev, origins in self._origins.items():
                for o in origins.values():
                    o.wait_stream(self._streams[dev])
            self.backward_joins = getattr(self, "backward_joins", 0) + 1

    def _issue_range(self, key, start, end, tag):
        torch = self._torch
        flat = self.groups[key]["flat"][start:end]
        side = self._side(key[1])
        if side is not None:
            cur = torch.cuda.current_stream(key[1])
            self._origins.setdefault(key[1], {})[cur.cuda_stream] = cur
            side.wait_stream(cur)
            ctx = torch.cuda.stream(side)
        else:
            import contextlib
            ctx = contextlib.nullcontext()
        with ctx:
            if self._average and self._passes > 1:
                flat.div_(self._passes)
            if end > start:
                self._issue_fn(flat)
        self.issue_log.append(tag)

    def _issue(self, b):
        key, s, e, _ = self.buckets[b]
        self._issue_range(key, s, e, b)
        self.issued[b] = True

    def synchronize(self, whole_groups=False):
        """Issue every bucket backward did not, in index order; the caller's streams then wait for
        the side streams. Returns the parameters whose gradient came sparse (for allreduce_grads).
        whole_groups=True (no backward ran on ANY rank since the last synchronize, so no bucket was
        issued anywhere): one allreduce per group instead of one per bucket."""
        torch = self._torch
        err = self.error
        with self._lock:
            for p in self.params:
                if id(p) not in self.seen:
                    self._adopt(p)  # no gradient: zeros; otherwise the view (copied in if needed)
            if whole_groups and any(self.issued):
                err = err or ("synchronize(whole_groups=True) after a backward that issued buckets: "
                              "the ranks' allreduces would not pair")
            whole = set()
            for b in range(self.next, len(self.buckets)):
                key = self.buckets[b][0]
                if whole_groups and not any(self.issued):
                    if key not in whole:
                        whole.add(key)
                        self._issue_range(key, 0, self.groups[key]["n"], ("group", key))
                elif not self.issued[b]:
                    self._issue(b)
            for dev, s in self._streams.items():
                torch.cuda.current_stream(dev).wait_stream(s)
            for p in self.params:
                if p.grad is not None and id(p) not in self.sparse:
                    v = self.view(p)
                    if p.grad.data_ptr() != v.data_ptr():
                        p.grad = v
            sparse = [p for p in self.params if id(p) in self.sparse]
            self.last_issue_log, self.issue_log = self.issue_log, []
            self._reset()
        if err:
            raise RuntimeError(err)
        return sparse


class _OverlapChoice(object):
    """Whether DistributedOptimizer's gradient buckets are allreduced during backward or after it,
    per optimizer step. mode "1" / "0": always / never. "auto": optimizer steps [W, W + 2M) alternate
    during / after (TIPS_OVERLAP_TRIAL_WARMUP W = 2 steps first, TIPS_OVERLAP_TRIAL_STEPS M = 3 of
    each), each step timed on the device from the end of the step before it to its own end (events
    on the caller's stream: forward, backward, the allreduces, the optimizer); after the last trial
    step every rank reports its mean per mode, the ranks take the slowest rank's (one small
    allgather, at the same step on every rank) and every rank keeps the faster mode from then on.
    The two modes issue the same bucket allreduces, so the trial changes no result."""

    def __init__(self, mode):
        import os
        self.mode = mode if mode in ("0", "1", "auto") else "auto"
        # at least 1: a trial step is timed from the end event of the step before it
        self.warm = max(1, int(os.environ.get("TIPS_OVERLAP_TRIAL_WARMUP", "2")))
        self.trials = max(1, int(os.environ.get("TIPS_OVERLAP_TRIAL_STEPS", "3")))
        self.chosen = {"0": False, "1": True}.get(self.mode)
        self.events = {}   # optimizer step -> event recorded at its end (trial window only)
        self.report = {"mode": self.mode}

    def on(self, s):
        """During backward for optimizer step s (0-based)?"""
        if self.chosen is not None:
            return self.chosen
        k = s - self.warm
        return k < 0 or k % 2 == 0  # (warm-up steps overlap, as round 3 did)

    def stepped(self, s):
        """After optimizer step s: time it (trial window) and decide after the last trial step."""
        if self.chosen is not None:
            return
        import torch
        if s >= self.warm - 1:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.events[s] = ev
        last = self.warm + 2 * self.trials - 1
        if s < last:
            return
        self.events[last].synchronize()
        per = {True: [], False: []}
        for t in range(self.warm, last + 1):
            per[self.on(t)].append(self.events[t - 1].elapsed_time(self.events[t]))
        mine = [int(sum(v) / len(v) * 1000) for v in (per[True], per[False])]  # us, during / after
        from .ops import _allgather_i64
        from . import basics
        allv = _allgather_i64(mine)
        n = basics.size()
        slow_on = max(allv[2 * r] for r in range(n))
        slow_off = max(allv[2 * r + 1] for r in range(n))
        self.chosen = slow_on < slow_off
        self.events = {}
        self.report.update(trial_steps_each=self.trials, during_backward_ms=slow_on / 1e3,
                           after_backward_ms=slow_off / 1e3, chosen="during" if self.chosen else "after")


class _DistributedOptimizer(object):
    """Wraps a torch.optim.Optimizer; step() allreduces the gradients first (__init__.py:252-335)."""

    def __init__(self, optimizer, compression, sparse_as_dense, op, backward_passes_per_step,
                 average_aggregated_gradients, groups):
        from . import Compression
        self._optimizer = optimizer
        self._compression = compression if compression is not None else Compression.none
        self._sparse_as_dense = sparse_as_dense
        self._op = op
        self._passes = int(backward_passes_per_step)
        self._average_aggregated = average_aggregated_gradients
        self._groups = groups
        self._calls = 0
        self._fused = {}  # (dtype, device, parameter ids) -> (ops.FusedList, flat buffer, offsets)
        import os
        self._bucket_view = os.environ.get("TIPS_GRAD_BUCKET_VIEW", "1") != "0"
        if self._passes < 1:
            raise ValueError("backward_passes_per_step must be >= 1")
        self._buckets = None
        # synchronize() bookkeeping: the step count and gradient-event count it ran at. step() skips
        # its own reduction only for a synchronize() of this very pass with no backward after it.
        self._sync_at = None
        self._grad_events = 0
        self._in_step = False
        from . import Compression
        self._overlap = _OverlapChoice(os.environ.get("TIPS_OVERLAP_BACKWARD", "auto").lower())
        if (self._overlap.mode != "0" and self._bucket_view
                and self._compression is Compression.none and not sparse_as_dense):
            import torch
            ps = [p for g in optimizer.param_groups for p in g["params"]
                  if p.requires_grad and p.is_cuda and p.layout == torch.strided
                  and p.dtype in (torch.float32, torch.float64, torch.float16, torch.bfloat16)]
            ps = list({id(p): p for p in ps}.values())  # (a parameter listed twice is one gradient)
            if ps:
                mib = float(os.environ.get("TIPS_GRAD_BUCKET_MIB", "25"))
                self._buckets = _GradBuckets(ps, max(1, int(mib * (1 << 20))), self._passes, self._average_aggregated)
                self._buckets.active = self._overlap_active
                self._buckets.final_pass = lambda: (self._calls + 1) % self._passes == 0
        import weakref
        ref = weakref.ref(self)

        def count(p, _ref=ref):
            o = _ref()
            if o is not None:
                o._grad_events += 1

        self._count_handles = [p.register_post_accumulate_grad_hook(count)
                               for p in {id(p): p for g in optimizer.param_groups for p in g["params"]
                                         if p.requires_grad}.values()]
        weakref.finalize(self, _remove_hooks, list(self._count_handles))

    def _overlap_active(self):
        """Hooks issue allreduces only once TiPS runs with more than one rank (never initialise
        TiPS from inside backward: synchronize() issues what the hooks did not), and only for a
        step _OverlapChoice runs during backward."""
        from . import basics
        return basics.is_initialized() and basics.size() > 1 and self._overlap.on(self._step_index())

    @property
    def overlap_choice(self):
        """{mode, and once decided: the trial's slowest-rank step means and the mode kept}."""
        return dict(self._overlap.report, current="during" if self._overlap.on(self._step_index()) else "after")

    # the wrapped optimizer's surface
    @property
    def param_groups(self):
        return self._optimizer.param_groups

    @property
    def state(self):
        return self._optimizer.state

    def zero_grad(self, set_to_none=True):
        return self._optimizer.zero_grad(set_to_none=set_to_none)

    def state_dict(self):
        return self._optimizer.state_dict()

    def load_state_dict(self, sd):
        return self._optimizer.load_state_dict(sd)

    def _params_with_grad(self):
        return [p for g in self._optimizer.param_groups for p in g["params"] if p.grad is not None]

    def synchronize(self, whole_groups=False):
        """Allreduce every parameter's .grad (compute_gradients, __init__.py:296-310).

        Dense contiguous device gradients without compression are summed IN PLACE: with gradient
        bucket views (default) as one allreduce of the flat buffer they are views of, no copies;
        with TIPS_GRAD_BUCKET_VIEW=0 through the fusion buckets (tips_fused_allreduce: pack, one
        allreduce per bucket, unpack straight back into .grad - 4 x the gradient bytes of HBM
        traffic). In a step run during backward (_GradBuckets at N > 1: TIPS_OVERLAP_BACKWARD=1, or
        auto's choice) most of that was issued during backward, and the end of backward already
        ordered the caller's stream after it; this issues the rest and joins, bucket by bucket (the
        same sequence on every rank whatever its hooks reached); in a step run after backward, one
        allreduce per group. whole_groups=True is for a caller that knows no
        backward ran on any rank since the last reduction (one allreduce per group).

        step() does not reduce again when the caller called synchronize() in the final pass of this
        step (to clip gradients, say) and no backward ran after it. A synchronize() in an earlier
        accumulation pass, or one followed by another backward (an evaluation that never stepped),
        does not excuse step(): it reduces, with a warning, as Horovod warns about synchronize()
        without skip_synchronize()."""
        from . import Compression, _fusable, allreduce_grads, size
        from .ops import FusedList
        if self._sync_at == (self._calls, self._grad_events):
            warnings.warn("DistributedOptimizer.synchronize() called again with no backward in between: "
                          "the gradients are reduced a second time")
        self._sync_at = (self._calls, self._grad_events)
        params = self._params_with_grad()
        if self._buckets is not None and size() > 1:
            # backward-overlapped buckets: the hooks issued what was ready; issue the rest in order.
            # A step _OverlapChoice runs after backward issued nothing on any rank (the choice is
            # the same on every rank): one allreduce per group's flat buffer instead of per bucket
            after = not self._overlap.on(self._step_index())
            sparse = set(id(p) for p in self._buckets.synchronize(whole_groups=whole_groups or after))
            managed = set(self._buckets.where)
            params = [p for p in params if id(p) not in managed or id(p) in sparse]
        if self._passes > 1 and self._average_aggregated:
            for p in params:
                p.grad = p.grad / self._passes
        if size() <= 1:  # _allreduce_cond: the identity on one rank (__init__.py:94-103)
            return
        inplace, rest = {}, []
        for p in params:
            g = p.grad
            if (self._compression is Compression.none and _fusable(g) and g.is_contiguous()
                    and not self._sparse_as_dense):
                inplace.setdefault((g.dtype, g.device), []).append(p)
            else:
                rest.append(p)
        for (dt, dev), group in inplace.items():
            # one FusedList per (dtype, device, parameter list): validated arrays reused while the
            # .grad tensors stay where they are (ops.FusedList)
            key = (dt, dev, tuple(id(p) for p in group))
            ent = self._fused.get(key)
            if ent is None:
                if len(self._fused) > 8:
                    self._fused.clear()
                numels = [p.numel() for p in group]
                flat, offs = None, []
                if self._bucket_view:
                    import torch
                    flat = torch.empty(sum(numels), dtype=dt, device=dev)
                    o = 0
                    for n in numels:
                        offs.append(o)
                        o += n
                ent = self._fused[key] = (FusedList(numels), flat, offs)
            fl, flat, offs = ent
            if flat is not None:
                # Gradient bucket views: every .grad becomes a view of one flat buffer, back to back,
                # and the flat buffer is allreduced in place as one tensor - no pack, no unpack. Its
                # size is the sum of the parameters' sizes, the same on every rank. A .grad that is
                # not (or no longer) its view - the first step, or after
                # zero_grad(set_to_none=True) - is copied in once; with set_to_none=False autograd
                # accumulates straight into the views.
                base, es = flat.data_ptr(), flat.element_size()
                for p, o in zip(group, offs):
                    g = p.grad
                    if g.data_ptr() != base + o * es:
                        v = flat[o:o + g.numel()].view_as(g)
                        v.copy_(g)
                        p.grad = v
                _allreduce_flat_(flat)
            else:
                fl.allreduce_([p.grad for p in group])
        if rest:
            reduced = allreduce_grads([p.grad for p in rest], compression=self._compression, op=self._op,
                                      sparse_as_dense=self._sparse_as_dense)
            for p, r in zip(rest, reduced):
                if r is not p.grad:
                    p.grad = r.to(p.grad.dtype) if (not r.is_sparse and r.dtype != p.grad.dtype) else r

    def step(self, closure=None):
        """Every backward_passes_per_step-th call: allreduce the (locally accumulated) gradients,
        then step the wrapped optimizer. Other calls only count (torch accumulates .grad across
        backward passes when zero_grad is not called in between), as the aggregation helper
        applies updates once per backward_passes_per_step (gradient_aggregation.py)."""
        self._calls += 1
        if self._calls % self._passes:
            return None
        sync_at, self._sync_at = self._sync_at, None
        if sync_at != (self._calls - 1, self._grad_events):
            if sync_at is not None:
                warnings.warn("DistributedOptimizer.synchronize() ran %s: step() reduces the gradients again"
                              % ("in an earlier accumulation pass" if sync_at[0] != self._calls - 1
                                 else "before a later backward"))
            self._in_step = True
            try:
                self.synchronize()
            finally:
                self._in_step = False
        self._sync_at = None
        out = self._optimizer.step(closure) if closure is not None else self._optimizer.step()
        if self._buckets is not None and self._overlap_ready():
            self._overlap.stepped(self._calls // self._passes - 1)
        return out

    def _step_index(self):
        """The optimizer step the gradients being reduced belong to: calls made so far // passes
        during backward (or a synchronize() before step()), one less inside step(), which has
        counted its own call already."""
        return (self._calls - (1 if self._in_step else 0)) // self._passes

    def _overlap_ready(self):
        from . import basics
        return basics.is_initialized() and basics.size() > 1


def _validate(op, gradient_predivide_factor, num_groups, groups):
    """The argument checks DistributedOptimizer and DistributedGradientTape share
    (__init__.py:408-423, 540-556), with the reference's messages; returns `groups`."""
    if gradient_predivide_factor != 1.0:
        if op != Average:
            raise ValueError('gradient_predivide_factor not supported with op != Average')
    if num_groups != 0:
        warnings.warn('Parameter `num_groups` has been replaced by `groups` '
                      'and will be removed in v0.23.0.', DeprecationWarning)
        if groups is None:
            groups = num_groups
    if groups is not None:
        if not (isinstance(groups, list) or groups > 0):
            raise ValueError('groups should be a non-negative integer or '
                             'a list of list of tf.Variable.')
    return groups


class _DistributedGradientTape(object):
    """gradient() computes the gradients, then sums them over the ranks
    (_DistributedGradientTape.gradient, __init__.py:485-488)."""

    def __init__(self, tape, compression, sparse_as_dense, op):
        from . import Compression
        self._tape = tape
        self._compression = compression if compression is not None else Compression.none
        self._sparse_as_dense = sparse_as_dense
        self._op = op

    def gradient(self, target, sources, output_gradients=None):
        from . import allreduce_grads
        single = not isinstance(sources, (list, tuple))
        srcs = [sources] if single else list(sources)
        if self._tape is not None:
            grads = self._tape.gradient(target, srcs, output_gradients)
        else:
            import torch
            grads = torch.autograd.grad(target, srcs, grad_outputs=output_gradients, allow_unused=True)
        reduced = allreduce_grads(list(grads), compression=self._compression, op=self._op,
                                  sparse_as_dense=self._sparse_as_dense)
        return reduced[0] if single else reduced


def DistributedGradientTape(gradtape=None,
                            device_dense='',
                            device_sparse='',
                            compression=None,
                            sparse_as_dense=False,
                            op=Average,
                            gradient_predivide_factor=1.0,
                            num_groups=0,
                            groups=None):
    """Same arguments and validation as the reference (__init__.py:490-569). torch has no tape
    object: with gradtape=None, gradient(target, sources, output_gradients) differentiates with
    torch.autograd.grad (allow_unused: a source the target does not depend on gets None, as
    tf.GradientTape returns); any object with that gradient() method can be wrapped instead.
    As for the optimizer, the gradients are SUMMED over ranks for op=Average too (__init__.py:82-87)."""
    _validate(op, gradient_predivide_factor, num_groups, groups)
    if gradtape is not None and not callable(getattr(gradtape, 'gradient', None)):
        raise ValueError('gradtape must have a gradient(target, sources, output_gradients) method: %s' % gradtape)
    return _DistributedGradientTape(gradtape, compression, sparse_as_dense, op)


def DistributedOptimizer(optimizer,
                         name=None,
                         use_locking=False,
                         device_dense='',
                         device_sparse='',
                         compression=None,
                         sparse_as_dense=False,
                         backward_passes_per_step=1,
                         op=Average,
                         gradient_predivide_factor=1.0,
                         average_aggregated_gradients=False,
                         num_groups=0,
                         groups=None):
    """Same arguments and validation as the reference (__init__.py:337-456); `optimizer` is a
    torch.optim.Optimizer. name / use_locking / device_* are accepted for signature compatibility."""
    groups = _validate(op, gradient_predivide_factor, num_groups, groups)
    try:
        import torch
        ok = isinstance(optimizer, torch.optim.Optimizer)
    except ImportError:  # pragma: no cover - torch is in the image
        ok = False
    if not ok:
        raise ValueError('Provided optimizer doesn\'t inherit from torch.optim.Optimizer: %s' % optimizer)
    return _DistributedOptimizer(optimizer, compression, sparse_as_dense, op, backward_passes_per_step,
                                 average_aggregated_gradients, groups)
