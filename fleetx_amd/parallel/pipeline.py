"""Pipeline parallelism: 1F1B and interleaved (virtual-stage) schedules.

Capability parity: Paddle ``PipelineLayer`` / ``PipelineParallel.train_batch``
/ ``PipelineParallelWithInterleave`` reached from reference
``eager_engine.py:400-410,521,577`` and ``hybrid_model.py:862-962`` (P05,
N10-N12): the local batch is split into ``accumulate_steps`` micro-batches;
warm-up forwards, steady 1F1B, cool-down backwards; activations / grads of
``[micro_b, s, h]`` move between neighbouring stages; the last stage computes
the loss (averaged over micro-batches) and the tied embedding grad is reduced
between the first and last stage.

MI355X design:
* stage-to-stage traffic uses ``batch_isend_irecv`` so a send and the
  opposite-direction receive of a 1F1B step are issued as ONE grouped RCCL
  p2p call (``ncclGroupStart/End``) -- no ordering deadlock, and both
  directions of the xGMI link are used at once;
* shapes are static (``[micro_b, s, h]`` in the model dtype), so there is no
  per-step shape handshake;
* gradient-bucket reductions of the flat grad buffer are armed only for the
  LAST backward of the step and overlap the cool-down phase.
"""
import torch
import torch.distributed as dist


class P2P:
    def __init__(self, hcg):
        self.hcg = hcg
        g = hcg.get_pipe_parallel_group()
        self.group = g.group if g is not None else None
        self.ranks = g.ranks if g is not None else [0]
        self.stage = hcg.pp_rank
        self.nstages = hcg.pp_degree
        self._warm = False

    def warmup(self, device):
        """One collective over the pipe group before the first grouped p2p
        call: RCCL/NCCL require every rank of the group to take part in the
        call that creates the communicator."""
        if not self._warm and self.group is not None and self.nstages > 1:
            t = torch.zeros(1, device=device)
            dist.all_reduce(t, group=self.group)
        self._warm = True

    def _peer(self, delta):
        return self.ranks[(self.stage + delta) % self.nstages]

    def _run(self, ops):
        if not ops:
            return
        reqs = dist.batch_isend_irecv(ops)
        for r in reqs:
            r.wait()

    def exchange(self, send_next=None, send_prev=None, recv_prev=None, recv_next=None):
        """Grouped p2p. ``recv_*`` are preallocated buffers (or None)."""
        ops = []
        if send_next is not None:
            ops.append(dist.P2POp(dist.isend, send_next.contiguous(), self._peer(1), self.group))
        if send_prev is not None:
            ops.append(dist.P2POp(dist.isend, send_prev.contiguous(), self._peer(-1), self.group))
        if recv_prev is not None:
            ops.append(dist.P2POp(dist.irecv, recv_prev, self._peer(-1), self.group))
        if recv_next is not None:
            ops.append(dist.P2POp(dist.irecv, recv_next, self._peer(1), self.group))
        self._run(ops)
        return recv_prev, recv_next


class PipelineSchedule:
    """Drives one training step over micro-batches for a stage model.

    ``stage_fn(chunk, micro_idx, x)`` runs model chunk ``chunk`` on micro-batch
    ``micro_idx`` (``x`` is the received activation or None on the first
    stage) and returns the activation, or the scaled loss on the last stage.
    """

    def __init__(self, hcg, act_shape_fn, dtype, device, num_chunks=1):
        self.p2p = P2P(hcg)
        self.hcg = hcg
        self.act_shape_fn = act_shape_fn
        self.dtype, self.device = dtype, device
        self.num_chunks = num_chunks
        self.p2p.warmup(device)

    def _buf(self):
        return torch.empty(self.act_shape_fn(), dtype=self.dtype, device=self.device)

    # ------------------------------------------------------------------ 1F1B
    def train_1f1b(self, m, stage_fn, on_last_backward=None):
        p2p = self.p2p
        first, last = p2p.stage == 0, p2p.stage == p2p.nstages - 1
        warmup = min(p2p.nstages - p2p.stage - 1, m)
        remaining = m - warmup
        ins, outs, losses = [], [], []
        n_bwd = [0]

        def fwd(k, x):
            if x is not None:
                x.requires_grad_(True)
            y = stage_fn(0, k, x)
            if last:
                losses.append(y.detach())
            return y

        def bwd(x, y, dy):
            n_bwd[0] += 1
            if n_bwd[0] == m and on_last_backward is not None:
                on_last_backward()
            if last:
                y.backward()
            else:
                torch.autograd.backward(y, dy)
            return x.grad if x is not None else None

        def recv_fwd():
            if first:
                return None
            return p2p.exchange(recv_prev=self._buf())[0]

        for k in range(warmup):
            x = recv_fwd()
            y = fwd(k, x)
            if not last:
                p2p.exchange(send_next=y.detach())
            ins.append(x)
            outs.append(y)
        x = recv_fwd() if remaining > 0 else None
        for k in range(remaining):
            y = fwd(warmup + k, x)
            ins.append(x)
            outs.append(y)
            dy = None
            if not last:
                dy = p2p.exchange(send_next=y.detach(), recv_next=self._buf())[1]
            xi, yo = ins.pop(0), outs.pop(0)
            dx = bwd(xi, yo, dy)
            if k == remaining - 1:
                x = None
                if not first:
                    p2p.exchange(send_prev=dx)
            else:
                if first:
                    x = None
                else:
                    x = p2p.exchange(send_prev=dx, recv_prev=self._buf())[0]
        for k in range(warmup):
            dy = None if last else p2p.exchange(recv_next=self._buf())[1]
            xi, yo = ins.pop(0), outs.pop(0)
            dx = bwd(xi, yo, dy)
            if not first:
                p2p.exchange(send_prev=dx)
        if last:
            return torch.stack(losses).sum()
        return None

    # ------------------------------------------------------------------ interleaved
    def train_interleaved(self, m, stage_fn, on_last_backward=None):
        """Interleaved 1F1B over ``num_chunks`` (V) virtual stages per rank.

        Virtual stage ``v = chunk * P + rank``; the last rank's chunk ``c``
        feeds rank 0's chunk ``c + 1``.  Unit ``u`` (of ``m * V``) runs chunk
        ``(u // P) % V`` on micro-batch ``(u // (P V)) P + u % P`` in forward,
        and the mirrored chunk in backward; the warm-up is
        ``2 (P - rank - 1) + (V - 1) P`` units.  Every p2p step posts the sends
        of this rank together with the receives it needs next in ONE grouped
        call, and the k-th send on a link always meets the k-th receive on the
        other side (the chunk shift on the ring edge is a +P unit shift, which
        preserves order), so the schedule cannot deadlock.  Requires
        ``m % P == 0``.
        """
        p2p = self.p2p
        P, V, r = p2p.nstages, self.num_chunks, p2p.stage
        assert m % P == 0, "interleaved schedule needs micro-batches % pp_degree == 0"
        total = m * V
        warmup = min((P - r - 1) * 2 + (V - 1) * P, total)
        remaining = total - warmup
        losses = []
        ins = [[] for _ in range(V)]
        outs = [[] for _ in range(V)]
        inputs = [[] for _ in range(V)]
        grads = [[] for _ in range(V)]
        n_bwd = [0]

        def fchunk(u):
            return (u // P) % V

        def bchunk(u):
            return V - 1 - (u // P) % V

        def micro(u):
            return (u // (P * V)) * P + u % P

        def first_v(c):
            return r == 0 and c == 0

        def last_v(c):
            return r == P - 1 and c == V - 1

        def forward(u):
            c = fchunk(u)
            x = None
            if not first_v(c):
                x = inputs[c].pop(0)
                x.requires_grad_(True)
            y = stage_fn(c, micro(u), x)
            ins[c].append(x)
            outs[c].append(y)
            if last_v(c):
                losses.append(y.detach())
                return None
            return y.detach()

        def backward(u):
            c = bchunk(u)
            x, y = ins[c].pop(0), outs[c].pop(0)
            n_bwd[0] += 1
            if n_bwd[0] == total and on_last_backward is not None:
                on_last_backward()
            if last_v(c):
                y.backward()
            else:
                torch.autograd.backward(y, grads[c].pop(0))
            if first_v(c):
                return None
            return x.grad

        def need_fwd_input(u):
            return u < total and not first_v(fchunk(u))

        def need_bwd_grad(u):
            return u < total and not last_v(bchunk(u))

        def exchange(send_next=None, send_prev=None, recv_for_fwd=None, recv_for_bwd=None):
            bp = self._buf() if recv_for_fwd is not None else None
            bn = self._buf() if recv_for_bwd is not None else None
            p2p.exchange(send_next=send_next, send_prev=send_prev, recv_prev=bp, recv_next=bn)
            if bp is not None:
                inputs[fchunk(recv_for_fwd)].append(bp)
            if bn is not None:
                grads[bchunk(recv_for_bwd)].append(bn)

        if need_fwd_input(0):
            exchange(recv_for_fwd=0)
        for u in range(warmup):
            y = forward(u)
            rf = u + 1 if need_fwd_input(u + 1) else None
            rb = 0 if (u == warmup - 1 and remaining > 0 and need_bwd_grad(0)) else None
            exchange(send_next=y, recv_for_fwd=rf, recv_for_bwd=rb)
        for k in range(remaining):
            uf, ub = warmup + k, k
            y = forward(uf)
            dx = backward(ub)
            rf = uf + 1 if need_fwd_input(uf + 1) else None
            rb = ub + 1 if need_bwd_grad(ub + 1) else None
            exchange(send_next=y, send_prev=dx, recv_for_fwd=rf, recv_for_bwd=rb)
        for ub in range(remaining, total):
            if ub == remaining and remaining == 0 and need_bwd_grad(ub):
                exchange(recv_for_bwd=ub)
            dx = backward(ub)
            rb = ub + 1 if need_bwd_grad(ub + 1) else None
            exchange(send_prev=dx, recv_for_bwd=rb)
        if r == P - 1:
            return torch.stack(losses).sum()
        return None

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def forward_only(self, m, stage_fn):
        p2p = self.p2p
        first, last = p2p.stage == 0, p2p.stage == p2p.nstages - 1
        losses = []
        for k in range(m):
            x = None if first else p2p.exchange(recv_prev=self._buf())[0]
            y = stage_fn(0, k, x)
            if last:
                losses.append(y.detach())
            else:
                p2p.exchange(send_next=y)
        if last:
            return torch.stack(losses).sum()
        return None
