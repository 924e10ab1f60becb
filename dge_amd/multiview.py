"""View-sharded data parallelism for the multi-view editing step.

The reference renders the views of a batch one after another on one GPU and
sums their gradients into the shared Gaussian parameters
(threestudio/systems/DGE.py:170-239 for the render loop, :266-296 for the
view-space gradient sum and the max-radii reduction).  It has no working
multi-GPU path.  Here each rank renders a contiguous shard
of the views (forward + backward through the gfx950 kernels) and ONE
collective per step sums the parameter gradients:

  * ``GradBucket`` makes every parameter's ``.grad`` a view into one flat
    fp32 buffer, so autograd accumulates straight into it and the step needs a
    single ``all_reduce`` (RCCL over xGMI with the ``nccl`` backend on ROCm;
    gloo in the CPU tests) with no pack/unpack copies;
  * the densification statistics the reference derives from the per-view
    renders (the sum of ``viewspace_points.grad`` and the max of ``radii``)
    reduce with one SUM and one MAX collective (``reduce_view_stats``).
Shard boundaries and the l1 mean's ``B_local / B`` factor keep the summed
gradient identical to the single-GPU loop up to summation order.
"""
from __future__ import annotations

from typing import Sequence

import ctypes
import weakref

import os

import torch
import torch.distributed as dist


def shard_views(num_views: int, world: int, rank: int) -> range:
    """Contiguous shard of view indices for `rank` (sizes differ by at most one)."""
    base, extra = divmod(num_views, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


# the dirty-row masks of the row-major GPU buckets, by their rows' address (the sparse all-reduce's scatter
# marks the rows it writes: _rows_scatter); DGE_AMD_SPARSE_ZERO=0 clears the whole bucket every zero()
_DIRTY_BY_ROWS = weakref.WeakValueDictionary()
_SPARSE_ZERO = os.environ.get("DGE_AMD_SPARSE_ZERO", "1") != "0"


class GradBucket:
    """One gradient buffer shared by a list of parameters.

    Row-major (``rows``, the default when every parameter has the same number of rows, as a GaussianModel's
    six do): one [n, pitch] fp32 matrix, every parameter's ``.grad`` a column block of it (a strided view,
    the parameter's shape), pitch = the summed row widths rounded up to 16 floats (59 -> 64 at SH degree 3)
    and 4-wide parameters (the rotation) first, on 16-byte boundaries.  A Gaussian's whole gradient is then
    one 256-B row: the per-Gaussian backward pass writes two cache lines per live Gaussian instead of one
    or two in each of six tensors (gs_grads.pitch_*), and the sparse all-reduce packs whole rows.
    Otherwise (``rows=False``, or parameters of different row counts) the flat concatenation."""

    def __init__(self, params: Sequence[torch.Tensor], rows: bool | None = None):
        self.params = list(params)
        dev = self.params[0].device
        n0 = {p.shape[0] if p.dim() else -1 for p in self.params}
        if rows is None:  # (GPU parameters: the fused backward writes the rows in place; autograd's own
            # accumulation into a strided .grad works too but warns about the layout contract)
            rows = (len(n0) == 1 and -1 not in n0 and all(p.dim() >= 1 and p.is_cuda for p in self.params))
        self.views = []
        self.rows = None
        if rows:
            n = n0.pop()
            widths = [p[0].numel() if n else int(torch.Size(p.shape[1:]).numel()) for p in self.params]
            order = sorted(range(len(self.params)), key=lambda i: widths[i] % 4 != 0)  # (stable: 4-wide first)
            cols, c = {}, 0
            for i in order:
                if widths[i] % 4 == 0:
                    c = (c + 3) // 4 * 4
                cols[i] = c
                c += widths[i]
            pitch = max(16, (c + 15) // 16 * 16)
            self._used = c  # (the columns a parameter owns: the sparse all-reduce packs only these)
            self.flat = torch.zeros(n * pitch, dtype=torch.float32, device=dev)
            self.rows = self.flat.view(n, pitch)
            if self.flat.is_cuda:  # (the rows written since the last zero(): a sparse clear, gs_rows_zero_dirty)
                self._dirty = torch.zeros(n, dtype=torch.uint8, device=dev)
                _DIRTY_BY_ROWS[self.rows.data_ptr()] = self._dirty
            for i, p in enumerate(self.params):
                self.views.append(self.rows[:, cols[i]:cols[i] + widths[i]].view(p.shape))
        else:
            total = sum(p.numel() for p in self.params)
            self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
            off = 0
            for p in self.params:
                self.views.append(self.flat[off:off + p.numel()].view_as(p))
                off += p.numel()
        self._rows_cap = 0       # speculated packed rows of the next sparse all-reduce (0: none yet)
        if not hasattr(self, "_dirty"):
            self._dirty = None
        self._deferred = None    # an allreduce_end(defer_check=True) awaiting allreduce_finalize()
        self.attach()

    def row_matrices(self):
        """The bucket as [n, width] matrices sharing their rows (the sparse all-reduce's regions), or None:
        the row-major matrix's used columns (59 of a GaussianModel's 64-float rows: the padding never
        travels), or each parameter's [n, -1] view of the flat layout."""
        if self.rows is not None:
            return [self.rows[:, :self._used]]
        rows = {v.shape[0] if v.dim() else -1 for v in self.views}
        n = next(iter(rows))
        return [v.reshape(n, -1) for v in self.views] if len(rows) == 1 and n >= 0 else None

    def attach(self):
        for p, v in zip(self.params, self.views):
            p.grad = v

    def zero(self, overlap: bool = False, stream=None, after=None):
        """Zero the bucket.  Default: on the current stream.  stream (GPU buckets): on that stream instead,
        after the event `after` (record it on the bucket's last user's stream — e.g. the default stream
        before the step's forwards are enqueued): the fused gradient writes of the next backward wait for
        the fill (gs_grads.writes_after), nothing else does, so the fill runs beside the step's forwards
        (dge_amd.multiview.render_views: pass one of the views' streams).  overlap: the round-2 form of the
        same, the fill on the current stream (measured no faster; with render_views the current stream
        already waits for the forwards).  For models on the fused raw-parameter path, whose gradients go
        into .grad in-kernel; a backward that hands its gradients to autograd's own accumulation must
        follow a plain zero()."""
        fixed = self.allreduce_finalize()  # (a deferred union check's fix-up writes the bucket: before the fill)
        # the previous step's packed scatter (or its fix-up) on a side stream still writes the bucket
        reduced, self._reduced = getattr(self, "_reduced", None), None
        self._zero_event = None
        if stream is not None and self.flat.is_cuda:
            from . import diff_gaussian_rasterization as _r

            dev = self.flat.device
            with torch.cuda.stream(stream):
                if after is not None:
                    stream.wait_event(after)
                if fixed:
                    stream.wait_stream(torch.cuda.current_stream(dev))
                if reduced is not None:
                    stream.wait_event(reduced)
                self._clear()
                self._zero_event = stream.record_event()
            _r._SIDE_STREAMS = True
            _r._GRAD_WRITES[dev.index] = (stream, self._zero_event)
            _r._ZEROED[dev.index] = (self.flat, self.flat._version)
            self.attach()
            return
        if reduced is not None:
            torch.cuda.current_stream(self.flat.device).wait_event(reduced)
        self._clear()
        if self.flat.is_cuda:
            from . import diff_gaussian_rasterization as _r

            _r._ZEROED[self.flat.device.index] = (self.flat, self.flat._version)
        if overlap and self.flat.is_cuda:
            from . import diff_gaussian_rasterization as _r

            dev = self.flat.device
            self._zero_event = torch.cuda.current_stream(dev).record_event()
            _r._SIDE_STREAMS = True
            _r._GRAD_WRITES[dev.index] = (torch.cuda.current_stream(dev), self._zero_event)
        self.attach()

    def _clear(self):
        """Zero the buffer on the current stream: only the rows written since the last clear when every writer
        since recorded them (the dirty-row record is intact: diff_gaussian_rasterization._DIRTY), else all of it;
        then a fresh record."""
        if self._dirty is None:
            self.flat.zero_()
            return
        from . import _native as N
        from . import diff_gaussian_rasterization as _r

        dev = self.flat.device
        rec = _r._DIRTY.get(dev.index)
        if rec is not None and rec[0] is self.flat and rec[2] == self.flat._version and _SPARSE_ZERO:
            n, pitch = self.rows.shape
            N.check(N.lib().gs_rows_zero_dirty(self.flat.data_ptr(), pitch, pitch, self._dirty.data_ptr(), n,
                                               torch.cuda.current_stream(dev).cuda_stream), "gs_rows_zero_dirty")
        else:
            self.flat.zero_()
            self._dirty.zero_()
        _r._DIRTY[dev.index] = [self.flat, self._dirty, self.flat._version]

    def _drop_dirty(self):
        """A write of every row not recorded in the dirty mask (a dense collective into the buffer)."""
        if self._dirty is not None:
            from . import diff_gaussian_rasterization as _r

            _r._DIRTY.pop(self.flat.device.index, None)

    def wait_zero(self):
        """Make the current stream wait for an overlapped zero() (no-op otherwise)."""
        ev = getattr(self, "_zero_event", None)
        if ev is not None:
            torch.cuda.current_stream(self.flat.device).wait_event(ev)

    def allreduce_begin(self, live_hint, group=None, min_world: int = 2, views=None):
        """First half of a sparse allreduce() whose union of live rows is agreed on BEFORE the backward runs,
        so the one host wait of the protocol (the union's size, which shapes the packed collective) waits
        for the forwards, not for the backward: call it after the views' forwards are enqueued and before
        backward(); allreduce_end() after the backward.

        live_hint: uint8 [rows] tensors, one per view rendered this step — render_views()' "_live_rows",
        the Gaussians some pixel of the view blends (set by the forward kernel), which are exactly the ones
        the backward gives a nonzero gradient row.  Valid only when the bucket was zeroed this step and
        these views' fused backward is the only writer of the gradients (the multi-view step); otherwise
        use allreduce(), which finds the nonzero rows by reading the bucket.

        views: the speculated batch these hints come from (render_views(speculate=True)'s list).  Its
        overflow flag (gs_views_overflow: some view outgrew its binning capacity, so its marks are not
        the re-rendered step's rows) travels with the marks in the same MAX, so every rank learns that
        SOME rank is re-rendering; allreduce_end then moves nothing at the agreed union and every rank
        runs the scanning allreduce() instead.  The rank that overflowed re-renders locally (no
        collective) between this call and allreduce_end — the same collectives on every rank."""
        self.allreduce_finalize()
        self._pending = None
        if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) < min_world:
            return
        mats = self.row_matrices()
        n = mats[0].shape[0] if mats is not None else -1
        hints = list(live_hint or [])
        if (mats is None or not hints or not _native_ok(mats)
                or any(h is None or h.dtype != torch.uint8 or h.shape != (n,) for h in hints)):
            self._pending = ("scan", group)  # no usable hint: allreduce() in allreduce_end
            return
        from . import _native as N

        dev = self.flat.device
        # on a side stream behind the forwards (which set the marks): the backward the caller enqueues
        # next on the current stream does not wait for the MAX collective and the compaction
        main = torch.cuda.current_stream(dev)
        side = _collective_stream(dev) if self.flat.is_cuda else main
        side.wait_stream(main)
        for h in hints:  # (read on the side stream; the caller may free the batch meanwhile)
            h.record_stream(side)
        batch = getattr(views, "batch", None)
        with torch.cuda.stream(side):
            live = torch.empty(n + 1, dtype=torch.uint8, device=dev)  # the rows' marks + the overflow flag
            live[:n].copy_(hints[0])
            for h in hints[1:]:
                live[:n] |= h
            if batch is not None:
                N.check(N.lib().gs_views_overflow(batch.handle, live[n:].data_ptr(), ctypes.c_void_p(side.cuda_stream)),
                        "gs_views_overflow")
            else:
                live[n:].zero_()
            dist.all_reduce(live, op=dist.ReduceOp.MAX, group=group)
            idx = torch.empty(n, dtype=torch.int64, device=dev)
            cs = torch.empty(1 + (n + 1023) // 1024, dtype=torch.int64, device=dev)
            N.check(N.lib().gs_rows_compact(live.data_ptr(), n, idx.data_ptr(), cs.data_ptr(),
                                            ctypes.c_void_p(side.cuda_stream)), "gs_rows_compact")
            # (count, agreed overflow flag); the device-side count of the packed collective is 0 when some
            # rank overflowed, so the speculated SUM moves nothing and the scanning allreduce() follows
            info = torch.cat([cs[:1], live[n:].to(torch.int64)])
            cdev = cs[:1] * (1 - info[1:])
            pinned = getattr(self, "_count_host", None)
            if pinned is None:
                pinned = self._count_host = torch.empty(2, dtype=torch.int64, pin_memory=True)
            pinned.copy_(info, non_blocking=True)
            ev = side.record_event()
        idx.record_stream(main)  # (read on the current stream by allreduce_end)
        cdev.record_stream(main)
        self._pending = ("hint", group, idx, pinned, ev, n, mats, cdev)

    def allreduce_end(self, stream=None, defer_check: bool = False):
        """Second half of allreduce_begin (after the backward): the packed SUM of the agreed rows.
        stream (GPU buckets): run the pack, the collective and the unpack on that stream instead, behind the
        work the current stream has enqueued so far (the backward), and return at once — the current stream
        is then free for work that does not read the gradients (DGE's gradient-free semantic renders,
        DGE.py:198-204) while RCCL runs; allreduce_join() makes the current stream wait for the result.
        defer_check (speculated capacity only): do not wait here for the union's size; the check (and the
        exact fix-up of rows past the capacity, in the rare step whose union outgrew it) runs in
        allreduce_finalize(), which the next zero() / allreduce_begin() / allreduce() / allreduce_join()
        call first — the caller finalizes before anything reads the gradients (an optimizer step)."""
        self.allreduce_finalize()
        pend, self._pending = getattr(self, "_pending", None), None
        if pend is None:
            return None
        if pend[0] == "scan":
            return self.allreduce(pend[1], min_world=1)
        _, group, idx, pinned, ev, n, mats, cs = pend
        main = torch.cuda.current_stream(self.flat.device)
        main.wait_event(ev)  # (idx and its count are written on the collective stream)
        self.wait_zero()
        if not self.check_attached():
            for p, v in zip(self.params, self.views):
                if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                    v.copy_(p.grad)
            self.attach()
        side = stream is not None and self.flat.is_cuda
        if side:
            stream.wait_stream(main)
            ctx = torch.cuda.stream(stream)
        else:
            import contextlib

            ctx = contextlib.nullcontext()
        # Speculative capacity: the union's size m shapes the packed collective, and reading it on the host
        # waits for the forwards (0.5 ms at the one-rank c2 step, the GPU that far behind).  With last
        # step's size as a capacity (+1/8), the gather / SUM / scatter of the first min(cap, m) rows is
        # enqueued with the count read on the device (gs_rows_gather_dev: zero rows past it, the same on
        # every rank), and only then does the host read m — the GPU has the backward and the collective
        # queued meanwhile.  m > cap (the union grew past the margin): the rows [cap, m) follow in a
        # second, exact packed SUM.  m is identical on every rank (the MAX-agreed union), so is cap.
        cap = getattr(self, "_rows_cap", 0)
        spec = 0 < cap and 2 * cap <= n
        with ctx:
            if spec:
                packed = _rows_gather(mats, idx, cap=cap, count=cs)
                dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
                _rows_scatter(mats, idx, packed, cap=cap, count=cs)
            if side:  # (allocated on the side stream, freed by the caching allocator at once)
                idx.record_stream(stream)
                cs.record_stream(stream)
            if spec and defer_check:
                self._deferred = (ev, pinned, cap, idx, group, mats, stream if side else None)
                self._reduced = stream.record_event() if side else None
                return None
            ev.synchronize()
            m, overflow = int(pinned[0]), int(pinned[1])
            if overflow:  # some rank re-rendered its views after the marks: every rank scans its bucket
                self.allreduce(group, min_world=1)
            elif spec:
                if m > cap:
                    _rows_fixup(mats, idx, cap, m, group)
            elif 2 * m > n:  # mostly dense: packing would not pay
                self._drop_dirty()  # (every row may change: the next zero() clears all of them)
                dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
            else:
                rows = idx[:m]
                packed = _rows_gather(mats, rows)
                dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
                _rows_scatter(mats, rows, packed)
        if not overflow:  # (an overflowed step's marks were abandoned: allreduce() set the cap from its scan)
            self._set_rows_cap(m, mats)
        self._reduced = stream.record_event() if side else None
        return None

    def _set_rows_cap(self, m, mats):
        self._rows_cap = m + m // 8 + 4096 if _native_ok(mats) and os.environ.get("DGE_AMD_ROWS_SPEC", "1") != "0" \
            else 0

    def allreduce_finalize(self) -> bool:
        """The deferred check of an allreduce_end(defer_check=True): wait for the union's size (the forwards'
        marks, long done by the next step), and when it exceeded the speculated capacity all-reduce the rows
        past it (exact; on the stream the packed SUM ran on).  Returns True when it enqueued that fix-up."""
        d, self._deferred = getattr(self, "_deferred", None), None
        if d is None:
            return False
        ev, pinned, cap, idx, group, mats, stream = d
        ev.synchronize()
        m, overflow = int(pinned[0]), int(pinned[1])
        if not overflow:  # (else allreduce() below sets the cap from the union it scans)
            self._set_rows_cap(m, mats)
        if m <= cap and not overflow:
            return False
        import contextlib

        with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            if overflow:  # (the packed SUM moved nothing: the agreed flag zeroed its device count)
                self.allreduce(group, min_world=1)
            else:
                _rows_fixup(mats, idx, cap, m, group)
            if stream is not None:
                self._reduced = stream.record_event()
        return True

    def allreduce_join(self):
        """Make the current stream wait for an allreduce_end(stream=...) (no-op otherwise)."""
        self.allreduce_finalize()
        ev, self._reduced = getattr(self, "_reduced", None), None
        if ev is not None:
            torch.cuda.current_stream(self.flat.device).wait_event(ev)

    def check_attached(self) -> bool:
        return all(p.grad is not None and p.grad.data_ptr() == v.data_ptr() for p, v in zip(self.params, self.views))

    def allreduce(self, group=None, async_op: bool = False, sparse: bool = True, min_world: int = 2):
        """SUM of the bucket over the ranks.  sparse (when every parameter has the same number of rows,
        as a GaussianModel's do): only rows that are nonzero on some rank travel — the union of the
        ranks' nonzero rows is agreed with one MAX all-reduce of a byte per row, those rows are packed,
        all-reduced and copied back.  A Gaussian behind saturated pixels in every view of every rank
        gets exactly zero gradient, so at c2 the union of 24 views is ~24% of the rows (~4x fewer
        bytes over xGMI than the dense 236 MB).  Rows outside the union are zero on every rank, so the
        result is the dense all-reduce's up to the float summation order inside RCCL.
        min_world: smallest group that communicates (1 runs the whole protocol on a one-rank group: the
        bench's RCCL rehearsal on a one-GPU box)."""
        self.allreduce_finalize()
        if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) < min_world:
            return None
        self.wait_zero()  # (a view whose backward wrote nothing still sees a zeroed bucket)
        if not self.check_attached():  # autograd replaced a grad: fold it back into the bucket
            for p, v in zip(self.params, self.views):
                if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                    v.copy_(p.grad)
            self.attach()
        mats = self.row_matrices()
        if not sparse or async_op or mats is None:
            self._drop_dirty()
            return dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
        n = mats[0].shape[0]
        live = _rows_live(mats, n)
        dist.all_reduce(live, op=dist.ReduceOp.MAX, group=group)
        idx = torch.nonzero(live).squeeze(1)
        self._set_rows_cap(int(idx.numel()), mats)  # (the next hinted step's speculated capacity)
        if 2 * idx.numel() > n:  # mostly dense: packing would not pay
            self._drop_dirty()
            return dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
        packed = _rows_gather(mats, idx)
        dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
        _rows_scatter(mats, idx, packed)
        return None


def _rows_fixup(mats, idx, cap, m, group):
    """The union's rows [cap, m) past a speculated capacity: their own exact packed SUM."""
    rows = idx[cap:m]
    packed = _rows_gather(mats, rows)
    dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
    _rows_scatter(mats, rows, packed)


# Sparse-row bookkeeping: one gfx950 kernel each on the GPU (gs_rows_live / gs_rows_gather /
# gs_rows_scatter, dge_amd/csrc/gs_bucket.hip); torch ops for CPU buckets (the gloo tests).
def _native_rows(mats):
    from . import _native as N

    regs = (N.RowsRegion * len(mats))(*[N.RowsRegion(m.data_ptr(), m.shape[1], m.stride(0) if m.shape[0] > 1 else 0) for m in mats])
    return N, regs, ctypes.c_void_p(torch.cuda.current_stream(mats[0].device).cuda_stream)


def _native_ok(mats):
    from . import _native as N

    return (mats[0].is_cuda and len(mats) <= N.ROWS_MAX_REGIONS
            and all(m.dtype == torch.float32 and m.dim() == 2 and (m.is_contiguous() or (
                m.stride(1) == 1 and m.stride(0) >= m.shape[1] and m.stride(0) < 2**31)) for m in mats))


def _rows_live(mats, n):
    """uint8 [n]: 1 where row r of some matrix has an element != 0."""
    live = torch.empty(n, dtype=torch.uint8, device=mats[0].device)
    if _native_ok(mats):
        N, regs, stream = _native_rows(mats)
        N.check(N.lib().gs_rows_live(regs, len(mats), n, live.data_ptr(), stream), "gs_rows_live")
        return live
    live.zero_()
    for m in mats:
        live |= (m != 0).any(1).to(torch.uint8)
    return live


def _rows_gather(mats, idx, cap=None, count=None):
    """[len(idx), sum(widths)]: the rows idx of every matrix, side by side.  cap/count (GPU): [cap, ...]
    holding the rows idx[:min(cap, count[0])] (count read on the device), zero rows after them."""
    if count is not None:
        N, regs, stream = _native_rows(mats)
        packed = torch.empty((cap, sum(m.shape[1] for m in mats)), dtype=torch.float32, device=mats[0].device)
        N.check(N.lib().gs_rows_gather_dev(regs, len(mats), idx.data_ptr(), cap, count.data_ptr(),
                                           packed.data_ptr(), stream), "gs_rows_gather_dev")
        return packed
    if _native_ok(mats):
        N, regs, stream = _native_rows(mats)
        packed = torch.empty((idx.numel(), sum(m.shape[1] for m in mats)), dtype=torch.float32,
                             device=mats[0].device)
        idx = idx.to(torch.int64).contiguous()
        N.check(N.lib().gs_rows_gather(regs, len(mats), idx.data_ptr(), idx.numel(), packed.data_ptr(), stream),
                "gs_rows_gather")
        return packed
    return torch.cat([m.index_select(0, idx) for m in mats], 1)


def _rows_scatter(mats, idx, packed, cap=None, count=None):
    """The inverse of _rows_gather: rows idx of every matrix = their columns of packed (and a row-major
    bucket's dirty-row mask records them)."""
    dirty = _DIRTY_BY_ROWS.get(mats[0].data_ptr()) if len(mats) == 1 and mats[0].is_cuda else None
    if count is not None:
        N, regs, stream = _native_rows(mats)
        N.check(N.lib().gs_rows_scatter_dev(regs, len(mats), idx.data_ptr(), cap, count.data_ptr(),
                                            packed.data_ptr(), stream), "gs_rows_scatter_dev")
        if dirty is not None:
            N.check(N.lib().gs_rows_mark_dirty(dirty.data_ptr(), idx.data_ptr(), cap, count.data_ptr(), stream),
                    "gs_rows_mark_dirty")
        return
    if _native_ok(mats):
        N, regs, stream = _native_rows(mats)
        idx = idx.to(torch.int64).contiguous()
        packed = packed.contiguous()
        N.check(N.lib().gs_rows_scatter(regs, len(mats), idx.data_ptr(), idx.numel(), packed.data_ptr(), stream),
                "gs_rows_scatter")
        if dirty is not None:
            N.check(N.lib().gs_rows_mark_dirty(dirty.data_ptr(), idx.data_ptr(), idx.numel(), None, stream),
                    "gs_rows_mark_dirty")
        return
    off = 0
    for m in mats:
        w = m.shape[1]
        m.index_copy_(0, idx, packed[:, off:off + w])
        off += w


_STREAM_POOLS = {}


def stream_pool(device, n: int):
    """n HIP streams of `device`, created once and reused."""
    dev = torch.device(device)
    key = (dev.index, n)
    pool = _STREAM_POOLS.get(key)
    if pool is None:
        from . import diff_gaussian_rasterization as _r

        _r._SIDE_STREAMS = True  # backward calls may now run off the default stream: order .grad writes
        pool = _STREAM_POOLS[key] = [torch.cuda.Stream(device=dev) for _ in range(n)]
    return pool


def view_streams(device, n: int):
    """The streams a batch of views runs on: the caller's current stream first (the first view, and the
    batch's merged per-Gaussian pass, need no cross-stream hop to or from the caller), then n - 1 pool
    streams.  (Three pool streams instead, the caller joining and forking around them: 2390 against 2500
    renders/s at c2, profiles/r03/bench_caller_first.txt.)"""
    main = torch.cuda.current_stream(device)
    if n <= 1:
        return [main]
    return [main] + stream_pool(device, n - 1)


def render_views(cameras, pc, pipe, bg_color, streams: int = 2, speculate: bool = False, **kw):
    """render() of every camera, the views spread round-robin over `streams` HIP streams.

    The reference renders a batch's views one after another (threestudio/systems/DGE.py:179-239) on
    one stream.  Here, for a standard GaussianModel (the fused raw-parameter path) and up to
    GS_MAX_VIEWS views, the batch goes through ONE autograd node over one native forward and one native
    backward (dge_amd.views): every view's first half is enqueued before any second half, consecutive
    views run on different streams (one view's latency-bound blend tail overlaps the others' work), and
    the backward chains the views' gradient accumulation in view order.  speculate: the views' binning
    buffers are sized from the instance counts seen before, without the per-view host wait for the count
    (rasterizer_impl.cu:236-239); the caller must then call `.check()` on the returned list before using
    the results (False: a view overflowed its capacity — render the batch again).  Other models: one
    render() per view on the pool's streams.  Returns a list (RenderedViews) of render()'s dicts,
    usable on the caller's stream."""
    from .gaussian_renderer import _fused_ok, render
    from .views import RenderedViews, render_views_batched

    dev = bg_color.device
    main = torch.cuda.current_stream(dev)
    if _fused_ok(pc, pipe) and 1 <= len(cameras) <= _native_max_views():
        return render_views_batched(cameras, pc, pipe, bg_color, view_streams(dev, streams), speculate=speculate,
                                    **kw)
    # (created only here: every stream takes one of the process's few hardware queues round-robin, and an
    # unused one can put a view's stream on the same queue as another's, serialising them)
    pool = stream_pool(dev, streams) if streams > 1 else [main]
    outs = RenderedViews()
    if len(pool) == 1:
        outs.extend(render(c, pc, pipe, bg_color, **kw) for c in cameras)
        return outs
    ready = main.record_event()
    for i, cam in enumerate(cameras):
        s = pool[i % len(pool)]
        s.wait_event(ready)
        with torch.cuda.stream(s):
            out = render(cam, pc, pipe, bg_color, **kw)
        for v in out.values():
            if isinstance(v, torch.Tensor) and v.is_cuda:
                v.record_stream(main)
        outs.append(out)
    for s in pool[:min(len(pool), len(cameras))]:
        main.wait_stream(s)
    return outs


_COLLECTIVE_STREAMS = {}


def _collective_stream(device):
    """The side stream a step's gradient collective runs on (one per device, reused)."""
    dev = torch.device(device)
    s = _COLLECTIVE_STREAMS.get(dev.index)
    if s is None:
        s = _COLLECTIVE_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    return s


def _native_max_views() -> int:
    from . import _native as N

    return N.MAX_VIEWS


def render_backward_views(cameras, pc, pipe, bg_color, grads, streams: int = 2, **kw):
    """Forward + backward of every view (d(image)/d(params) contracted with `grads[i]`, accumulated into
    the parameters' .grad), view i on stream i % `streams`: view i's backward overlaps view i+1's
    forward.  The gradients equal the reference's batch step (all views rendered, one backward of the
    summed loss) up to float summation order.  Returns the render() dicts with the images detached."""
    from .gaussian_renderer import render

    dev = bg_color.device
    main = torch.cuda.current_stream(dev)
    pool = stream_pool(dev, streams) if streams > 1 else [main]
    ready = main.record_event()
    outs = []
    for i, (cam, g) in enumerate(zip(cameras, grads)):
        s = pool[i % len(pool)]
        if s != main:
            s.wait_event(ready)
        with torch.cuda.stream(s):
            out = render(cam, pc, pipe, bg_color, **kw)
            out["render"].backward(g)
        out = {k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}
        if s != main:
            for v in out.values():
                if isinstance(v, torch.Tensor) and v.is_cuda:
                    v.record_stream(main)
        outs.append(out)
    for s in pool[:min(len(pool), len(cameras))]:
        if s != main:
            main.wait_stream(s)
    return outs


def reduce_view_stats(viewspace_grad_sum: torch.Tensor, radii_max: torch.Tensor, group=None):
    """SUM of the view-space gradient accumulator, MAX of radii across ranks (in place)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(viewspace_grad_sum, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(radii_max, op=dist.ReduceOp.MAX, group=group)
    return viewspace_grad_sum, radii_max


def found_inf_allreduce(bucket: GradBucket, group=None) -> torch.Tensor:
    """1 if any gradient of this rank's bucket is inf/NaN on SOME rank, else 0 (a MAX all-reduce of one
    flag), computed before the gradient all-reduce: Lightning's 16-mixed GradScaler (configs/dge.yaml:81)
    skips the optimizer step on overflow, and every replica must skip the same steps or their
    parameters diverge.  (The SUM all-reduce would spread an inf/NaN to every rank anyway — for the
    rows it carries; this flag makes the decision explicit and independent of the sparse packing.)"""
    flag = (~torch.isfinite(bucket.flat)).any().to(torch.float32).reshape(1)  # (after or before the SUM)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    return flag


def multiview_step(scene, cameras, render_fn, pipe, bg, bucket: GradBucket, total_views: int, targets=None,
                   gt_images=None, masks=None, lambda_l1: float = 1.0, loss_scale: float = 1.0,
                   semantic: bool = False, group=None, streams: int = 1, bucket_zeroed: bool = False,
                   min_world: int = 2):
    """One data-parallel step of DGE's edit loop over this rank's views (threestudio/systems/DGE.py
    forward :170-239, training_step :617-699, on_before_optimizer_step :266-296).

    The per-view loss is either a given gradient seed (``targets[i]`` = dL/dimage, [3,H,W]) or DGE's
    l1 term: ``F.l1_loss(images * mask, gt * mask)`` is a mean over all B views' elements
    (DGE.py:672), so this rank's share is its views' absolute-error SUM over (B * H * W * 3) — the
    local mean times B_local / B — and the ranks' gradients add up to the single-GPU loop's.
    (The perceptual term, :673-676, is a per-view ``.sum()``: unchanged under sharding; its network is
    out of scope.)  ``loss_scale`` is the GradScaler's scale (16-mixed); ``semantic`` also runs DGE's
    mask render per view (:198-204, override_color = the Gaussian mask) — gradient-free, so here
    without autograd, its boolean ``norm > 0.8`` map returned in ``masks``.

    Then one (sparse-row) SUM all-reduce of the gradient bucket, the overflow flag (any non-finite
    gradient of the reduced bucket on some rank: one MAX all-reduce, found_inf_allreduce), and the
    densification statistics: the SUM of the view-space gradients and the MAX of the radii across views
    and ranks.  Returns a dict: viewspace_grad_sum [P,3], radii_max [P], found_inf (float tensor [1]),
    semantic_masks (list of [H,W] bool, when ``semantic``).

    streams > 1 with this package's render (dge_amd.gaussian_renderer.render): the views are rendered
    together (render_views: one autograd node, the views on that many HIP streams) and ONE backward of
    their summed loss follows — the reference's order (DGE.py renders the batch, then back-propagates).
    With ``bucket_zeroed`` (the caller zeroed the bucket this step and these losses are the only gradient
    source): the views' binning buffers are speculated (no per-view host wait; the batch is checked after
    the backward and the step redone in the rare case a view overflowed), and the all-reduce's union of
    live rows is agreed on between the forwards and that backward (GradBucket.allreduce_begin), so the
    host does not wait for the backward before the collective is shaped.  The semantic renders are issued
    after the collective, so they overlap it.
    """
    from .gaussian_renderer import render as _render

    P = scene.num_points()
    dev = bucket.flat.device
    vs_sum = torch.zeros((P, 3), dtype=torch.float32, device=dev)
    radii_max = torch.zeros((P,), dtype=torch.int32, device=dev)
    sem = []
    batched = streams > 1 and render_fn is _render and len(cameras) > 1

    def losses_of(pkgs, first=0):
        out = []
        for i, pkg in enumerate(pkgs, first):
            img = pkg["render"]
            if targets is not None:
                loss = (img * targets[i]).sum()
            else:
                m = masks[i] if masks is not None else torch.ones_like(img[:1])
                loss = torch.abs(img * m - gt_images[i] * m).sum() * (lambda_l1 / (total_views * img.numel()))
            out.append(loss * loss_scale if loss_scale != 1.0 else loss)
        return out

    hinted = False
    if batched:
        def attempt(begin):
            pkgs = render_views(cameras, scene, pipe, bg, streams=streams, speculate=bucket_zeroed)
            ok = bucket_zeroed and all("_live_rows" in pkg for pkg in pkgs)
            if begin and ok:
                bucket.allreduce_begin([pkg["_live_rows"] for pkg in pkgs], group, min_world=min_world, views=pkgs)
            torch.autograd.backward(losses_of(pkgs))
            return pkgs, ok

        pkgs, hinted = attempt(True)
        if not pkgs.check():
            # this rank's speculated capacity overflowed (speculated only with bucket_zeroed): render and
            # back-propagate again locally, no collective — the overflow flag the union's MAX carried makes
            # every rank's allreduce_end re-agree on the rows by scanning the buckets
            bucket.zero()
            pkgs, _ = attempt(False)
            if not pkgs.check():
                raise RuntimeError("multiview_step: the binning capacity check failed twice")
        for pkg in pkgs:
            vs_sum += pkg["viewspace_points"].grad
            radii_max = torch.maximum(radii_max, pkg["radii"])
    else:
        for i, cam in enumerate(cameras):
            pkg = render_fn(cam, scene, pipe, bg)
            losses_of([pkg], i)[0].backward()
            vs_sum += pkg["viewspace_points"].grad
            radii_max = torch.maximum(radii_max, pkg["radii"])
    side = None
    if hinted:
        # the collective on a side stream behind the backward; the semantic renders (which read no
        # gradient) go on the caller's stream meanwhile, and the caller's stream joins the collective after
        side = _collective_stream(dev) if semantic and dev.type == "cuda" else None
        bucket.allreduce_end(stream=side)
    else:
        bucket.allreduce(group, min_world=min_world)
    if semantic:  # gradient-free: beside the collective (hinted steps) or behind it
        with torch.no_grad():
            gm = getattr(scene, "mask", None)
            gm = gm if gm is not None else torch.ones(P, dtype=torch.bool, device=dev)
            colors = gm[..., None].float().repeat(1, 3)
            if batched:
                sms = [o["render"] for o in render_views(cameras, scene, pipe, bg, streams=streams,
                                                         override_color=colors)]
            else:
                sms = [render_fn(cam, scene, pipe, bg, override_color=colors)["render"] for cam in cameras]
            sem = [torch.norm(sm, dim=0) > 0.8 for sm in sms]
    bucket.allreduce_join()
    # (the explicit MAX of every rank's flag: a non-finite element outside the all-reduced rows still
    # makes every rank skip the step)
    found_inf = found_inf_allreduce(bucket, group)
    reduce_view_stats(vs_sum, radii_max, group)
    out = {"viewspace_grad_sum": vs_sum, "radii_max": radii_max, "found_inf": found_inf}
    if semantic:
        out["semantic_masks"] = sem
    return out
