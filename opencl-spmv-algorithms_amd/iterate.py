"""iterate.py — iterated SpMV over row shards: power iteration and CG.

SURVEY.md §8f row 3: "Iterated SpMV (power iteration / CG) reusing the y
all-gather as the next x".  The reference stops after one SpMV (reference
csr.c:198-236: launch, read y back, check), so this module has no reference
counterpart; it is the natural consumer of the row-sharded design of §8e.

Layout.  Rank r owns rows [bounds[r], bounds[r+1]) (spmv_partition_rows,
nnz-balanced).  The vector that multiplies A is kept in the GATHERED layout:
`world` blocks of `pad` entries, block r = rank r's rows followed by zeros.
The shard's column indices are renumbered into that layout once, at build
time, so `all_gather_into_tensor` of each rank's padded block IS the next
x — no reorder pass, and the y all-gather becomes the input
of the next SpMV directly.

Overlap (build_operator(..., overlap=True), world > 1).  The shard is
split by column into a LOCAL part (columns in this rank's own block, which
it already holds) and a REMOTE part (every other column).  One step of
A·x then starts the all-gather of the own block (RCCL runs it on its own
stream), runs the local SpMV on the compute stream while the exchange is in
flight, waits, runs the remote SpMV into a scratch y and adds it
(spmv_axpy_ratio with ratio 1: an exact add).  overlap=False with split=True
runs the same launches with the wait first, so the two produce the same
bits; the split itself regroups each row's sum (local entries, then
remote) and so differs from the unsplit SpMV within the parity rule.

Per iteration everything stays on the device: SpMV (libspmv_hip), the
deterministic dot product, and the vector updates read their scalars
(norms, CG's alpha = rr/pAp and beta = rr'/rr) from device memory; the
scalars are all-reduced in place over RCCL (`torch.distributed`, backend
nccl) and never visit the host except for CG's convergence test every
`check_every` iterations.  With one rank the loop can be captured into a
HIP graph (`graph=True`).

The device work goes through a `kernels` object (HipKernels by default).
Tests substitute a numpy double to exercise the multi-rank orchestration on
CPU ranks (gloo); the product path only ever builds HipKernels.
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass

import numpy as np

import spmv_amd as sa


# ------------------------------------------------------------------ layout
@dataclass
class ShardLayout:
    """Row ownership and the gathered vector layout for `world` ranks."""

    bounds: np.ndarray  # int64[world + 1]
    pad: int  # entries per rank in the gathered vector

    @property
    def world(self) -> int:
        return len(self.bounds) - 1

    def positions(self, idx: np.ndarray) -> np.ndarray:
        """Gathered-layout position of global row/column indices."""
        idx = np.asarray(idx, np.int64)
        owner = np.searchsorted(self.bounds, idx, side="right") - 1
        return (owner * self.pad + (idx - self.bounds[owner])).astype(np.int64)

    def to_gathered(self, v: np.ndarray) -> np.ndarray:
        out = np.zeros(self.world * self.pad, dtype=v.dtype)
        out[self.positions(np.arange(len(v)))] = v
        return out

    def from_gathered(self, g: np.ndarray, n: int) -> np.ndarray:
        return np.asarray(g)[self.positions(np.arange(n))]


def layout_for(n_rows: int, row_counts: np.ndarray, world: int, align: int = 1024) -> ShardLayout:
    """nnz-balanced row ranges (spmv_partition_rows) and a pad rounded up to
    64 entries (one wave of x per block)."""
    ptr = np.zeros(n_rows + 1, np.int64)
    np.cumsum(row_counts, out=ptr[1:])
    bounds = sa.partition_rows(n_rows, ptr, world, align)
    pad = int(np.max(np.diff(bounds))) if world > 0 else 0
    pad = max(64, (pad + 63) // 64 * 64)
    return ShardLayout(bounds, pad)


def local_shard(m: sa.Coo, layout: ShardLayout, rank: int) -> sa.Coo:
    """Rank `rank`'s rows with columns renumbered into the gathered layout
    (square matrices: x and y share the row partition)."""
    if m.n_rows != m.n_cols:
        raise sa.SpmvError(sa.OTHER_ERROR, "local_shard", "iterated SpMV needs a square matrix")
    lo, hi = int(layout.bounds[rank]), int(layout.bounds[rank + 1])
    loc = sa.shard(m, lo, hi)
    col = layout.positions(loc.col)
    if col.size and col.max() > np.iinfo(np.int32).max:
        raise sa.SpmvError(sa.OTHER_ERROR, "local_shard", "gathered layout exceeds int32 columns")
    return sa.Coo(hi - lo, layout.world * layout.pad, loc.row, col.astype(np.int32), loc.val, m.symmetric,
                  f"{m.label} rank {rank}/{layout.world}")


def split_local_remote(loc: sa.Coo, layout: ShardLayout, rank: int):
    """(local, remote) parts of a gathered-layout shard: `local` keeps the
    entries whose column lies in this rank's own block, renumbered to
    [0, pad) so it multiplies the rank's send block directly; `remote` keeps
    the rest with gathered-layout columns.  Both keep all the shard's rows
    and their entries in the shard's order."""
    base = rank * layout.pad
    own = (loc.col >= base) & (loc.col < base + layout.pad)
    local = sa.Coo(loc.n_rows, layout.pad, loc.row[own], (loc.col[own] - base).astype(np.int32), loc.val[own],
                   False, f"{loc.label} local")
    remote = sa.Coo(loc.n_rows, loc.n_cols, loc.row[~own], loc.col[~own], loc.val[~own], False,
                    f"{loc.label} remote")
    return local, remote


# ------------------------------------------------------------- collectives
class Comm:
    """In-place collectives over torch.distributed (nccl = RCCL on ROCm);
    with one rank they are no-ops and the gathered vector aliases the local
    block."""

    def __init__(self, dist=None):
        self.dist = dist if dist is not None and dist.is_available() and dist.is_initialized() else None
        self.rank = self.dist.get_rank() if self.dist else 0
        self.world = self.dist.get_world_size() if self.dist else 1

    def allreduce(self, t) -> None:
        if self.dist is not None and self.world > 1:
            self.dist.all_reduce(t)

    def allgather(self, out, inp) -> None:
        if self.dist is not None and self.world > 1:
            self.dist.all_gather_into_tensor(out, inp)
        elif out.data_ptr() != inp.data_ptr():
            out[: inp.numel()].copy_(inp)

    def allgather_start(self, out, inp):
        """Start the all-gather; returns a handle for wait() (None when
        alone: the copy is done at once)."""
        if self.dist is not None and self.world > 1:
            return self.dist.all_gather_into_tensor(out, inp, async_op=True)
        if out.data_ptr() != inp.data_ptr():
            out[: inp.numel()].copy_(inp)
        return None

    @staticmethod
    def wait(work, stream=None) -> None:
        """Make the compute stream wait for a started collective (NCCL: a
        stream dependency, the host does not block).  work.wait() orders
        torch's CURRENT stream only; when the kernels run on another
        `stream`, that stream waits on an event recorded on the current one
        behind the collective."""
        if work is None:
            return
        work.wait()
        if stream is not None:
            torch = sa._torch()
            cur = torch.cuda.current_stream(stream.device)
            if cur.cuda_stream != stream.cuda_stream:
                ev = torch.cuda.Event()
                ev.record(cur)
                stream.wait_event(ev)

    def allgatherv(self, full, bounds) -> str:
        """In-place all-gather of row shards of their REAL sizes: `full`
        holds this rank's rows [bounds[rank], bounds[rank+1]) and receives
        every other rank's, no padding to the largest shard.  Over RCCL one
        torch all_gather of unequal parts (ProcessGroupNCCL issues it as
        grouped broadcasts, one per shard); over gloo one broadcast per
        non-empty shard.  Returns how it was done."""
        if self.dist is None or self.world == 1:
            return "none (one rank)"
        parts = [full[int(bounds[r]):int(bounds[r + 1])] for r in range(self.world)]
        if self.dist.get_backend() == "nccl":
            self.dist.all_gather(parts, parts[self.rank])
            return "rccl all_gather of unequal parts (grouped broadcasts)"
        for r in range(self.world):
            if parts[r].numel():
                self.dist.broadcast(parts[r], src=r)
        return "gloo broadcast per shard"


# ---------------------------------------------------------------- kernels
class HipKernels:
    """The device kernels of one iteration, all on one stream."""

    def __init__(self, dm: sa.DeviceMatrix, stream=None):
        torch = sa._torch()
        self.dm = dm
        self.dev = torch.device(dm.device)
        self.lib = sa.hip_lib()
        self.stream = stream

    def _s(self):
        torch = sa._torch()
        st = self.stream if self.stream is not None else torch.cuda.current_stream(self.dev)
        return st.cuda_stream

    def spmv(self, x_full, y) -> None:
        self.dm.run(x_full, y, self.stream)

    def dot(self, n, a, b, out, ws) -> None:
        sa._check(self.lib.spmv_dot(n, sa._ptr(a), sa._ptr(b), sa._ptr(out), sa._ptr(ws), ws.numel(),
                                    self.dev.index or 0, self._s()), "spmv_dot")

    def axpy_ratio(self, n, num, den, sign, x, y) -> None:
        sa._check(self.lib.spmv_axpy_ratio(n, sa._ptr(num), sa._ptr(den), float(sign), sa._ptr(x), sa._ptr(y),
                                           self.dev.index or 0, self._s()), "spmv_axpy_ratio")

    def xpay_ratio(self, n, num, den, x, y) -> None:
        sa._check(self.lib.spmv_xpay_ratio(n, sa._ptr(num), sa._ptr(den), sa._ptr(x), sa._ptr(y),
                                           self.dev.index or 0, self._s()), "spmv_xpay_ratio")

    def scale_rsqrt(self, n, s, x, y) -> None:
        sa._check(self.lib.spmv_scale_rsqrt(n, sa._ptr(s), sa._ptr(x), sa._ptr(y), self.dev.index or 0,
                                            self._s()), "spmv_scale_rsqrt")

    def dot_ws(self, n):
        torch = sa._torch()
        nbytes = self.lib.spmv_dot_ws_bytes(n)
        return torch.empty(nbytes, dtype=torch.uint8, device=self.dev)


# --------------------------------------------------------------- operator
@dataclass
class DistOperator:
    """One rank's share of a square matrix in the gathered layout."""

    layout: ShardLayout
    rank: int
    n: int  # global rows
    kernels: object  # HipKernels (or a test double); the LOCAL part when split
    device: object = None
    remote: object = None  # kernels of the remote-column part (split shards only)
    overlap: bool = False  # split shards: run the local part while the all-gather is in flight

    @property
    def world(self) -> int:
        return self.layout.world

    @property
    def lo(self) -> int:
        return int(self.layout.bounds[self.rank])

    @property
    def rows(self) -> int:
        return int(self.layout.bounds[self.rank + 1] - self.layout.bounds[self.rank])

    @property
    def pad(self) -> int:
        return self.layout.pad


def build_operator(m: sa.Coo, rank: int = 0, world: int = 1, fmt: str = "csr", device="cuda:0", align: int = 1024,
                   split: bool = False, overlap: bool = False, **fmt_kw) -> DistOperator:
    """Partition, renumber and upload this rank's shard (HIP kernels).
    split (implied by overlap): local / remote column parts
    (split_local_remote), each its own device matrix."""
    counts = np.bincount(m.row, minlength=m.n_rows).astype(np.int64)
    layout = layout_for(m.n_rows, counts, world, align)
    loc = local_shard(m, layout, rank)
    if not (split or overlap):
        return DistOperator(layout, rank, m.n_rows, HipKernels(sa.to_device(loc, fmt, device, **fmt_kw)), device)
    local, remote = split_local_remote(loc, layout, rank)
    return DistOperator(layout, rank, m.n_rows, HipKernels(sa.to_device(local, fmt, device, **fmt_kw)), device,
                        HipKernels(sa.to_device(remote, fmt, device, **fmt_kw)), overlap)


def _zeros(op, n):
    torch = sa._torch()
    return torch.zeros(n, dtype=torch.float64, device=op.device)


class _Apply:
    """y = A·x for the vector whose own block is `send` (gathered into
    `full` by this call).  Unsplit: all-gather, then one SpMV on `full`.
    Split: start the all-gather, local SpMV on `send` (before or after the
    wait: overlap), wait, remote SpMV on `full` into a scratch vector, exact
    add."""

    def __init__(self, op, comm, full, send):
        self.op, self.comm, self.full, self.send = op, comm, full, send
        if op.remote is not None:
            self.y2 = _zeros(op, max(op.rows, 1))
            self.one = _zeros(op, 1) + 1.0

    def __call__(self, y) -> None:
        op, comm = self.op, self.comm
        st = getattr(op.kernels, "stream", None)
        cur = sa._torch().cuda.current_stream(st.device) if st is not None else None
        # the collective (or the one-rank copy) runs on torch's current
        # stream and reads `send`, which the kernels' stream produced: order
        # it behind them (both directions)
        _order(st, cur)
        if op.remote is None:
            comm.allgather(self.full, self.send)
            _order(cur, st)
            op.kernels.spmv(self.full, y)
            return
        work = comm.allgather_start(self.full, self.send)
        if work is None:
            _order(cur, st)  # one rank: the copy was queued on the current stream
        if not op.overlap:
            comm.wait(work, st)
        op.kernels.spmv(self.send, y)  # own block only: runs while the exchange is in flight
        comm.wait(work, st)
        op.remote.spmv(self.full, self.y2)
        op.kernels.axpy_ratio(op.rows, self.one, self.one, 1.0, self.y2, y)  # y += y_remote, exact


def _order(src, dst) -> None:
    """dst waits for the work queued on src so far (no-op for one stream)."""
    if src is None or dst is None or src.cuda_stream == dst.cuda_stream:
        return
    ev = sa._torch().cuda.Event()
    ev.record(src)
    dst.wait_event(ev)


def _gathered_pair(op, comm):
    """(full gathered vector, this rank's send block); one tensor when alone."""
    if comm.world > 1:
        return _zeros(op, op.world * op.pad), _zeros(op, op.pad)
    full = _zeros(op, op.pad)
    return full, full


# -------------------------------------------------------- power iteration
def _kernel_stream(op):
    """Context that makes the operator's kernel stream torch's current one
    for a whole solve, so torch copies, host reads and the collectives are
    ordered with the HIP kernels; no-op on the default stream."""
    st = getattr(op.kernels, "stream", None)
    return sa._torch().cuda.stream(st) if st is not None else contextlib.nullcontext()


def power_iteration(op: DistOperator, iters: int, comm: Comm | None = None, x0=None, graph: bool = False,
                    block: int = 16):
    """x <- A x / ||A x||, `iters` times, on the operator's kernel stream
    (_power_iteration has the details)."""
    with _kernel_stream(op):
        return _power_iteration(op, iters, comm, x0, graph, block)


def _power_iteration(op: DistOperator, iters: int, comm: Comm | None = None, x0=None, graph: bool = False,
                     block: int = 16):
    """x <- A x / ||A x||, `iters` times.  Returns (hist, x_local): hist is a
    host array [iters, 2] of (x·Ax, ||Ax||²) per iteration — x·Ax converges
    to the dominant eigenvalue of a symmetric A — and x_local is this
    rank's block of the final normalised x (device).  graph=True (one rank)
    replays `block` iterations per HIP graph launch; same kernels, same
    bits."""
    torch = sa._torch()
    comm = comm or Comm()
    k = op.kernels
    rows = op.rows
    full, send = _gathered_pair(op, comm)
    x_loc = send[:rows]
    if x0 is None:  # deterministic start, no zero entries, not orthogonal to much
        gidx = np.arange(op.lo, op.lo + rows)
        x_loc.copy_(torch.from_numpy(1.0 + (gidx % 7) / 7.0))
    else:
        x_loc.copy_(x0)
    ws = k.dot_ws(rows)
    s0 = _zeros(op, 1)
    k.dot(rows, x_loc, x_loc, s0, ws)
    comm.allreduce(s0)
    k.scale_rsqrt(rows, s0, x_loc, x_loc)
    y = _zeros(op, max(rows, 1))
    hist = _zeros(op, 2 * max(iters, 1)).view(-1, 2)
    apply = _Apply(op, comm, full, send)

    def step(h):
        apply(y)  # gathers x (overlapped with the local part when split)
        k.dot(rows, x_loc, y, h[0:1], ws)
        k.dot(rows, y, y, h[1:2], ws)
        comm.allreduce(h)  # both scalars in one collective
        k.scale_rsqrt(rows, h[1:2], y, x_loc)

    done = 0
    if graph and comm.world == 1 and iters > block:
        # one eager step (first-call setup), then `block` steps per graph
        # replay: 7 launches per step become one graph launch per block
        step(hist[0])
        done = 1
        blk = _zeros(op, 2 * block).view(-1, 2)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for j in range(block):
                step(blk[j])
        while done + block <= iters:
            g.replay()
            hist[done:done + block].copy_(blk)
            done += block
    for it in range(done, iters):
        step(hist[it])
    return hist[:iters].cpu().numpy(), x_loc


# ---------------------------------------------------------------------- CG
def cg(op: DistOperator, b_loc, comm: Comm | None = None, tol: float = 1e-10, maxit: int = 1000,
       check_every: int = 10):
    """Conjugate gradients on the operator's kernel stream (_cg)."""
    with _kernel_stream(op):
        return _cg(op, b_loc, comm, tol, maxit, check_every)


def _cg(op: DistOperator, b_loc, comm: Comm | None = None, tol: float = 1e-10, maxit: int = 1000,
        check_every: int = 10):
    """Conjugate gradients for a symmetric positive definite A, x0 = 0.
    Returns (x_local, iterations, relative residual ||r||/||b||)."""
    comm = comm or Comm()
    k = op.kernels
    rows = op.rows
    full, send = _gathered_pair(op, comm)
    p = send[:rows]
    x = _zeros(op, rows)
    r = b_loc.clone()
    p.copy_(b_loc)
    apply = _Apply(op, comm, full, send)
    Ap = _zeros(op, max(rows, 1))
    ws = k.dot_ws(rows)
    rr, rr_new, pAp = _zeros(op, 1), _zeros(op, 1), _zeros(op, 1)
    k.dot(rows, r, r, rr, ws)
    comm.allreduce(rr)
    bb = float(rr.item())
    if bb == 0.0:
        return x, 0, 0.0
    it = 0
    while it < maxit:
        apply(Ap)  # gathers p (overlapped with the local part when split)
        k.dot(rows, p, Ap, pAp, ws)
        comm.allreduce(pAp)
        k.axpy_ratio(rows, rr, pAp, 1.0, p, x)  # x += alpha p
        k.axpy_ratio(rows, rr, pAp, -1.0, Ap, r)  # r -= alpha Ap
        k.dot(rows, r, r, rr_new, ws)
        comm.allreduce(rr_new)
        k.xpay_ratio(rows, rr_new, rr, r, p)  # p = r + beta p
        rr, rr_new = rr_new, rr
        it += 1
        if it % check_every == 0 or it == maxit:
            if float(rr.item()) <= tol * tol * bb:
                break
    return x, it, float(np.sqrt(max(float(rr.item()), 0.0) / bb))
