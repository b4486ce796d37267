"""Multi-GPU harness for the engine: one process per GPU,
independent channels/streams sharded across ranks with no data-path
collective -- or one long FIR / decimator stream time-sharded, each rank
reading its segment plus a halo of preceding inputs -- max-over-ranks timing,
and an RCCL gather of results to rank 0 after the timed region.

Backend-agnostic on purpose: bench.py runs it over RCCL ("nccl") with device
tensors; tests/test_parallel_gloo.py runs the same functions over gloo with
CPU tensors at world size 2.
"""
from __future__ import annotations

import os


def world():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(total: int, world_size: int, rank: int) -> list[int]:
    """Round-robin shard of `total` independent channels: rank r gets r, r+W, r+2W, ..."""
    if world_size < 1 or not (0 <= rank < world_size):
        raise ValueError("bad rank / world size")
    return list(range(rank, total, world_size))


def channel_ids(per_rank: int, world_size: int, rank: int) -> list[int]:
    """Weak scaling: every rank owns `per_rank` channels; global ids rank*per_rank + s."""
    return [rank * per_rank + s for s in range(per_rank)]


def max_over_ranks(value: float, device=None) -> float:
    """The job's time is the slowest rank's (all_reduce MAX); a no-op without a process group (an
    initialised group of one rank still runs the collective: bench.py --dist)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_to_root(piece, root: int = 0):
    """Gather one equally-shaped tensor per rank onto `root` (list on root, None elsewhere)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [piece]
    rank = dist.get_rank()
    bufs = [torch.empty_like(piece) for _ in range(dist.get_world_size())] if rank == root else None
    dist.gather(piece.contiguous(), bufs, dst=root)
    return bufs


def gather_full_to_root(out, root: int = 0, chunk_bytes: int = 1 << 30):
    """Gather every rank's whole 1-D output onto `root` as one [world, numel]
    tensor (None on the other ranks).  The transfer is cut into chunks of at
    most `chunk_bytes` per rank, each one `gather` straight into the row
    slices of the result (no staging copy), so RCCL moves large messages
    point to point over the root's xGMI links.  Every rank passes the same numel."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return out.reshape(1, -1)
    world, rank = dist.get_world_size(), dist.get_rank()
    out = out.reshape(-1)
    if not out.is_contiguous():
        raise ValueError("gather_full_to_root: output must be contiguous")
    cplx = out.is_complex()
    if cplx:  # neither gloo nor RCCL gathers complex dtypes: move the interleaved (re, im) pairs as reals
        out = torch.view_as_real(out).reshape(-1)
    numel = out.numel()
    step = max(1, chunk_bytes // out.element_size())
    if cplx:
        step -= step % 2  # a chunk never splits a (re, im) pair
        step = max(step, 2)
    big = torch.empty((world, numel), dtype=out.dtype, device=out.device) if rank == root else None
    for c0 in range(0, numel, step):
        c1 = min(numel, c0 + step)
        dist.gather(out[c0:c1], [big[r, c0:c1] for r in range(world)] if rank == root else None, dst=root)
    if cplx and big is not None:
        big = torch.view_as_complex(big.view(world, numel // 2, 2))
    return big


# ---------------------------------------------------------------------------
# Checking a gathered output (bench.py after the RCCL gather; the gloo dry run).
# The index arithmetic lives here, testable without a GPU; the expected values
# come from a caller-supplied function (bench.py passes the f64 restatement).

def fir_input_window(s: int, width: int, taps: int):
    """Inputs that determine FIR outputs [s, s + width) of a stream (y[n] uses
    x[n - taps + 1 .. n], fir/mod.rs:209-212): (first input, input count, outputs of
    a zero-state run over them to drop).  Needs s >= taps - 1."""
    if s < taps - 1:
        raise ValueError("window starts before the first full delay line")
    return s - (taps - 1), width + taps - 1, taps - 1


def decim_input_window(m: int, width: int, taps: int, M: int):
    """Inputs that determine decimated outputs [m, m + width) of a stream that started
    at phase 0 (y[m] uses x[(m+1)M - 1 - i], i < taps; decim.rs:221-228): (first input,
    input count); the outputs are the zero-state dot products of the length-`taps`
    windows starting every M inputs.  Needs (m+1)M >= taps."""
    first = (m + 1) * M - taps
    if first < 0:
        raise ValueError("window starts before the first full delay line")
    return first, (width - 1) * M + taps


def check_gathered(big, expected, rng, width: int, lo: int, hi: int, windows: int = 2) -> float:
    """Worst relative RMS error over `windows` random output windows [s, s + width),
    lo <= s <= hi - width, of every row of a gathered [ranks, n] output (row r =
    channel r), against expected(r, s, width)."""
    import numpy as np
    worst = 0.0
    rows = big.shape[0]
    for r in range(rows):
        for _ in range(windows):
            s = int(rng.integers(lo, hi - width + 1))
            ref = np.asarray(expected(r, s, width), dtype=np.complex128)
            got = big[r, s:s + width]
            got = got.cpu().numpy() if hasattr(got, "cpu") else np.asarray(got)
            got = np.asarray(got, dtype=np.complex128)
            if got.shape != ref.shape:
                return float("inf")
            worst = max(worst, float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-300)))
    return worst


# ---------------------------------------------------------------------------
# Time-sharding one long stream: rank r filters the global inputs
# [r n, (r + 1) n) of a single stream.  A FIR output depends on the L - 1 inputs
# before it only, so the rank first feeds `halo` preceding inputs to a fresh
# handle (their outputs are dropped) and its outputs are then exactly the single
# stream's; no exchange.  A decimator's halo is a multiple of M, so the fresh
# handle's phase lines up with the global one (segments start at multiples of M).

def fir_halo(taps: int) -> int:
    """inputs a FIR segment reads before its own (the delay line, fir/mod.rs:209-212)"""
    return taps - 1


def decim_halo(taps: int, M: int) -> int:
    """the delay line rounded up to whole decimation periods (decim.rs:221-228): the
    fresh handle's phase 0 falls on a global multiple of M"""
    return -(-(taps - 1) // M) * M


def time_segment(n: int, rank: int, halo: int):
    """(first global input the rank reads, halo inputs actually read): rank 0 starts
    the stream from the zero state, so it reads no halo"""
    h = min(halo, rank * n)
    return rank * n - h, h


def check_time_sharded(big, expected, rng, width: int, lo: int, windows: int = 2) -> float:
    """Worst relative RMS error of the gathered outputs of one time-sharded stream
    ([ranks, m] rows, row r = global outputs [r m, (r + 1) m)) against
    expected(global_first_output, width): `windows` random windows inside every row
    (global index >= lo), and one window across every boundary between two rows --
    where a wrong halo or phase would show."""
    import numpy as np
    rows, m = big.shape[0], big.shape[1]
    flat = big.reshape(-1)
    starts = []
    for r in range(rows):
        a = max(lo, r * m)
        for _ in range(windows):
            starts.append(int(rng.integers(a, (r + 1) * m - width + 1)))
        if r > 0:
            starts.append(r * m - width // 2)
    worst = 0.0
    for g in starts:
        ref = np.asarray(expected(g, width), dtype=np.complex128)
        got = flat[g:g + width]
        got = np.asarray(got.cpu().numpy() if hasattr(got, "cpu") else got, dtype=np.complex128)
        if got.shape != ref.shape:
            return float("inf")
        worst = max(worst, float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-300)))
    return worst


# ---------------------------------------------------------------------------
# Time-sharding one IIR stream ("one exchange step: an exclusive scan of
# the 2 S-dim boundary state").  The SOS cascade carries D = 2 S state values across
# a cut -- (w1, w2) of every section, src/filter/iir/sos.rs:92-114, in the device
# handle's layout -- so segments are not independent.  Rank r runs its segment
# x[r n, (r + 1) n) from zero state (outputs y0_r, final state s_r); the ranks
# exchange the s_r (one all_gather of D values each); every rank forms the exclusive
# scan  I_0 = st0,  I_{r+1} = Phi I_r + s_r  with Phi = A^n (the state transition
# over one segment), and adds the zero-input response of its true initial state:
#     y_r[i] = y0_r[i] + c A^i I_r,
# computed by a second handle set to state I_r over i < W zeros, where W is where
# c A^i has decayed below rounding (the whole segment when it does not decay).
# Exact up to rounding for every cascade, decaying or not; the exchange is D values.

def sos_state_space(ff, fb):
    """(A, b, c, d) of an SOS cascade in f64, state S = [w1_0, w2_0, w1_1, w2_1, ...]:
    S' = A S + b x, y = c S + d x, with the coefficients normalised by a0 as
    SecondOrderFilter::new does (sos.rs:55-75) and the recurrence of sos.rs:92-114
    (section q feeds section q + 1, iir/mod.rs:281-287)."""
    import numpy as np
    ff = np.asarray(ff, np.float64).reshape(-1, 3)
    fb = np.asarray(fb, np.float64).reshape(-1, 3)
    S = len(ff)
    D = 2 * S

    def step(st, x):
        st = st.copy()
        v = x
        for q in range(S):
            a0 = fb[q, 0]
            b0, b1, b2 = ff[q] / a0
            a1, a2 = fb[q, 1] / a0, fb[q, 2] / a0
            w1, w2 = st[2 * q], st[2 * q + 1]
            w = v - (a1 * w1 + a2 * w2)
            v = b0 * w + b1 * w1 + b2 * w2
            st[2 * q + 1] = w1
            st[2 * q] = w
        return st, v

    A = np.zeros((D, D))
    c = np.zeros(D)
    for j in range(D):
        e = np.zeros(D)
        e[j] = 1.0
        A[:, j], c[j] = step(e, 0.0)
    b, d = step(np.zeros(D), 1.0)
    return A, b, c, d


def state_transition(A, n: int):
    """A^n in f64 by repeated squaring"""
    import numpy as np
    R = np.eye(A.shape[0])
    P = np.array(A, np.float64)
    while n:
        if n & 1:
            R = P @ R
        P = P @ P
        n >>= 1
    return R


def iir_exclusive_scan(states, Phi, st0=None):
    """I_0 = st0 (zero state when None), I_{r+1} = Phi I_r + states[r]: the true initial
    state of every segment from the segments' zero-state final states"""
    import numpy as np
    D = Phi.shape[0]
    cur = np.zeros(D, dtype=np.result_type(np.asarray(states).dtype, np.float64)) if st0 is None else \
        np.asarray(st0, dtype=np.result_type(np.asarray(st0).dtype, np.float64))
    out = []
    for s in states:
        out.append(cur.copy())
        cur = Phi @ cur + np.asarray(s)
    return out


def zero_input_length(A, c, n: int, rel: float = 1e-12) -> int:
    """samples after which the zero-input response c A^i I is below `rel` of its peak gain
    (rounded up to 4096, at most n); n when it does not decay within n samples"""
    import numpy as np
    g = np.array(c, np.float64)
    peak = max(np.abs(g).sum(), 1e-300)
    i = 0
    while i < n:
        if np.abs(g).sum() <= rel * peak and i > 0:
            return min(n, -(-i // 4096) * 4096)
        g = g @ A
        i += 1
        peak = max(peak, np.abs(g).sum())
    return n


def exchange_states(state, device=None):
    """all_gather of every rank's D-value state (complex as (re, im) pairs) in f64: the
    one collective of the IIR time shard"""
    import numpy as np
    import torch
    import torch.distributed as dist
    s = np.asarray(state)
    cplx = np.iscomplexobj(s)
    flat = np.stack([s.real, s.imag], -1).reshape(-1) if cplx else s.astype(np.float64)
    t = torch.tensor(np.asarray(flat, np.float64), device=device)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        parts = [t]
    else:
        parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, t)
    out = [p.cpu().numpy() for p in parts]
    if cplx:
        out = [o.reshape(-1, 2) @ np.array([1.0, 1.0j]) for o in out]
    return out
