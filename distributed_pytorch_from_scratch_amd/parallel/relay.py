"""TP = 2 collectives routed over every xGMI link of the node (two-hop relays).

An 8 x MI355X node is a fully connected xGMI mesh: one point-to-point link from every GPU to
each of its 7 peers.  A TP = 2 group (the ``BASELINE.json`` GPT-2-small layout, scaled out by
data parallelism: ``tp2dp4`` on 8 GPUs) has exactly ONE link between its two GPUs, so every
reduce-scatter / all-gather of the Megatron-SP step serialises on it while the other six links
of each GPU idle (they only carry the per-step DP gradient buckets).  At d = 768 that link, not
the MFMA work, sets the step time (README "Known limits").

``RelayComm`` spreads each pair's exchange over all links.  The payload one rank sends its
partner (half of the reduce-scatter input / the all-gather input) is cut into R + 2 units
(R = world - 2 relays): two units go over the direct link, and one unit goes to each relay GPU,
which forwards it to the partner in a second hop.  Every TP pair runs the same collective at
the same time (SPMD), so each GPU also relays one unit of each of the other pairs' two
directions.  Per link and direction the load is then 2 units = 1/4 of the direct-only payload
at W = 8 (1/2 at W = 4): link a->k carries a's unit for its partner plus the unit a forwards
to k for k's partner, and the direct link a->b carries a's two direct units.

Both hops are batched point-to-point groups (``dist.batch_isend_irecv``) on the WORLD process
group (RCCL ``ncclSend`` / ``ncclRecv`` inside one ``ncclGroupStart/End`` each), issued from a
high-priority side stream that waits for the producer; the second hop waits for the first on
that side stream only, so neither the host nor the compute stream blocks until the handle is
waited.  The reduce-scatter sum (own half + the partner's contribution) runs on the caller's
stream at that point.  A relay forwards unit j of x's payload, where j is its position in x's
sorted relay list; x's partner expects unit j from the relay at position j of ITS list, which is
the same set (every rank but the two of the pair) in the same order.  Because every rank of the WORLD takes part in every relayed collective,
``parallel/tp_comm.py`` only selects this transport by a WORLD-wide decision (validated against
the RCCL sum and timed against RCCL / xGMI on every rank), never per group.

Message sizes: a relay receives a unit from every other pair, so every pair must cut its payload
with the SAME unit size.  Two pairs of a ``tp2dpN`` layout hold different batches, and real-data
batches are padded per batch, so their payloads can differ.  Unless the caller declared fixed
shapes (``tp_comm.set_fixed_shapes``: synthetic data / fixed-length batches, the only case
``auto`` offers this transport for), every exchange first agrees on the WORLD-wide maximum
payload (one tiny all-reduce) and pads to it; the receiver keeps its own pair's prefix.
"""
from __future__ import annotations

from typing import List

import torch
import torch.distributed as dist


class _RelayWork:
    """Completion handle: waits the second hop, then (reduce-scatter) adds the own half."""

    def __init__(self, works: List, finish=None, keep=()):
        self.works, self.finish, self.keep = works, finish, keep

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []
        if self.finish is not None:
            self.finish()
            self.finish = None
        self.keep = ()
        return True


class RelayComm:
    def __init__(self, p):
        assert p.tp_size == 2, "relayed collectives are for TP = 2 pairs"
        W = dist.get_world_size()
        assert W >= 4 and W % 2 == 0, "relays need at least one other TP pair on the node"
        self.world = W
        self.rank = dist.get_rank()
        grid = p.grid.tolist()
        self.partner_of = {}
        for row in grid:
            a, b = int(row[0]), int(row[1])
            self.partner_of[a], self.partner_of[b] = b, a
        self.partner = self.partner_of[self.rank]
        self.tp_rank = p.tp_rank
        # my relays (every rank but me and my partner) = my partner's relays, same order
        self.relays = sorted(r for r in range(W) if r not in (self.rank, self.partner))
        # the ranks I relay for (the members of every other pair)
        self.sources = list(self.relays)
        self.R = len(self.relays)
        self._side = None
        # gloo moves CUDA tensors by their raw device pointers from host threads, outside any
        # stream order (single-GPU multi-rank rehearsals only): fence it with device syncs
        self._host_fence = dist.get_backend() == "gloo"
        # payload sizes are WORLD-uniform (set by tp_comm from set_fixed_shapes); otherwise
        # every exchange agrees on the WORLD maximum first and pads to it
        self.fixed_shapes = False

    # ---------------------------------------------------------------- exchange core ----
    def _split(self, n: int):
        """(direct elements, relay unit elements): n = direct + R * q, direct >= 2q."""
        q = (n // (self.R + 2)) // 8 * 8
        return n - self.R * q, q

    def _world_max(self, n: int) -> int:
        t = torch.tensor([n], dtype=torch.int64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item())

    def _exchange(self, payload: torch.Tensor, recv: torch.Tensor) -> List:
        """recv <- the partner's payload (same numel: the two ranks of a pair always agree).
        Pads to the WORLD-wide maximum payload first unless shapes are declared fixed."""
        n = payload.numel()
        N = n if self.fixed_shapes else self._world_max(n)
        if N == n:
            return self._exchange_n(payload, recv)
        pay_p = payload.new_zeros(N)
        pay_p[:n].copy_(payload)
        recv_p = recv.new_empty(N)
        works = self._exchange_n(pay_p, recv_p)
        return works + [_CopyBack(recv, recv_p[:n], keep=pay_p)]

    def _exchange_n(self, payload: torch.Tensor, recv: torch.Tensor) -> List:
        """recv <- the partner's payload (same numel), direct units + relayed units.
        Returns the works of the second hop (or of the only hop when nothing is relayed).

        On the GPU both hops are issued from a side stream that first waits for the caller's
        stream (the producer of ``payload``); the second hop waits for the first on that side
        stream only, so the caller's stream keeps running until it waits on the handle."""
        n = payload.numel()
        d, q = self._split(n)
        P = dist.P2POp
        side = None
        if payload.is_cuda:
            if self._side is None:
                self._side = torch.cuda.Stream(priority=-1)
            side = self._side
            side.wait_stream(torch.cuda.current_stream())
        fence = self._host_fence and payload.is_cuda
        ctx = torch.cuda.stream(side) if side is not None else _nullctx()
        with ctx:
            if fence:
                torch.cuda.synchronize()
            ops = [P(dist.isend, payload[:d], self.partner), P(dist.irecv, recv[:d], self.partner)]
            relay_buf = None
            if q > 0:
                relay_buf = payload.new_empty(len(self.sources), q)
                for j, k in enumerate(self.relays):
                    ops.append(P(dist.isend, payload[d + j * q: d + (j + 1) * q], k))
                for i, x in enumerate(self.sources):
                    ops.append(P(dist.irecv, relay_buf[i], x))
            works = dist.batch_isend_irecv(ops)
            if q == 0:
                return works + ([_Fence()] if fence else [])
            # hop 2 reads relay_buf: the first hop must have landed (side-stream order on the
            # GPU, a host wait for gloo's CPU transport)
            for w in works:
                w.wait()
            if fence:
                torch.cuda.synchronize()
            ops = []
            for i, x in enumerate(self.sources):
                ops.append(P(dist.isend, relay_buf[i], self.partner_of[x]))
            for j, k in enumerate(self.relays):
                ops.append(P(dist.irecv, recv[d + j * q: d + (j + 1) * q], k))
            works = dist.batch_isend_irecv(ops)
        # relay_buf is read by the second hop: it lives until the caller's wait on the handle
        return works + [_Hold(relay_buf)] + ([_Fence()] if fence else [])

    # ----------------------------------------------------------------- collectives ----
    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = True):
        """out = (inp + partner's inp)[tp_rank-th half] (``dist.reduce_scatter_tensor`` contract)."""
        assert inp.numel() == 2 * out.numel()
        halves = inp.contiguous().view(2, -1)
        mine, theirs = halves[self.tp_rank], halves[1 - self.tp_rank]
        recv = torch.empty_like(mine)
        works = self._exchange(theirs, recv)
        o = out.view(-1)

        def finish():
            torch.add(mine, recv, out=o)
        h = _RelayWork(works, finish, keep=(halves, recv))
        if not async_op:
            h.wait()
            return None
        return h

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = True):
        """out = concat(rank 0's inp, rank 1's inp) of the pair (``all_gather_into_tensor``)."""
        assert out.numel() == 2 * inp.numel()
        halves = out.view(2, -1)
        src = inp.contiguous().view(-1)
        halves[self.tp_rank].copy_(src)
        works = self._exchange(src, halves[1 - self.tp_rank])
        h = _RelayWork(works, keep=(src,))
        if not async_op:
            h.wait()
            return None
        return h

    def all_reduce(self, t: torch.Tensor, async_op: bool = True):
        """In-place SUM over the pair: relayed reduce-scatter, then relayed all-gather, both
        ordered on the side stream (the caller's stream only waits on the returned handle)."""
        flat = t.view(-1)
        if flat.numel() % 2:
            # odd count: sum a zero-padded copy (every rank pads the same way, so the call
            # sequence stays WORLD-uniform; no per-rank fallback to another transport)
            padded = flat.new_zeros(flat.numel() + 1)
            padded[:-1].copy_(flat)
            h = self.all_reduce(padded, async_op=True)
            cb = _RelayWork([h, _CopyBack(flat, padded[:-1])])
            if not async_op:
                cb.wait()
                return None
            return cb
        if flat.is_cuda:
            if self._side is None:
                self._side = torch.cuda.Stream(priority=-1)
            self._side.wait_stream(torch.cuda.current_stream())
            flat.record_stream(self._side)
        ctx = torch.cuda.stream(self._side) if flat.is_cuda else _nullctx()
        with ctx:
            half = flat.new_empty(flat.numel() // 2)
            self.reduce_scatter(half, flat, async_op=False)
            h = self.all_gather(flat, half, async_op=True)
        if not async_op:
            h.wait()
            return None
        return h


class _CopyBack:
    """Completion step of a padded exchange: the pair's own prefix of the padded receive
    buffer goes to the caller's tensor (after every hop has been waited)."""

    def __init__(self, dst, src, keep=None):
        self.dst, self.src, self.keep = dst, src, keep

    def wait(self):
        if self.src is not None:
            self.dst.view(-1).copy_(self.src)
        self.src = self.keep = None
        return True


class _Hold:
    """Keeps a tensor an in-flight transfer reads alive until the handle is waited."""

    def __init__(self, t):
        self.t = t

    def wait(self):
        self.t = None
        return True


class _Fence:
    """Device sync after gloo's host-side transfers into CUDA tensors (rehearsal path)."""

    def wait(self):
        torch.cuda.synchronize()
        return True


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False
