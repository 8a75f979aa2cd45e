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
* grouped ``batch_isend_irecv`` calls (``ncclGroupStart/End``) on one RCCL
  communicator per pipe group by default -- an in-order stream that is
  deadlock-free whatever hardware queue it lands in; with
  ``Distributed.comm.pp_split_directions`` activations (stage s -> s+1, and
  the ring edge of the interleaved schedule) and gradients (s+1 -> s) get a
  communicator each, so a gradient never queues behind an activation (needs
  ``GPU_MAX_HW_QUEUES`` >= the peer-waiting streams, ``utils/streams.py``);
* nothing waits for a SEND: the compute stream only waits for a receive, and
  only where the received tensor is consumed (``_Recv.wait``).  Posting the
  receive of the next micro-batch's input together with the current send lets
  the transfer run under the backward pass that follows.  (With NCCL/RCCL a
  ``Work.wait`` is a stream-level wait, not a host block.)  Pending sends are
  retired at the end of the step;
* the split is deadlock-free by construction: per direction, the k-th send on
  a link meets the k-th receive on the other side, and separating the
  directions / deferring waits only REMOVES ordering edges from the original
  single-stream schedule;
* shapes are static (``[micro_b, s, h]`` in the model dtype), so there is no
  per-step shape handshake;
* gradient-bucket reductions of the flat grad buffer are armed only for the
  LAST backward of the step and overlap the cool-down phase.
"""
import torch
import torch.distributed as dist


class _Recv:
    """A posted receive: ``wait()`` orders the consumer after the transfer and
    returns the buffer."""

    __slots__ = ("buf", "works")

    def __init__(self, buf, works):
        self.buf, self.works = buf, works

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = ()
        return self.buf


class P2P:
    def __init__(self, hcg):
        self.hcg = hcg
        g = hcg.get_pipe_parallel_group()
        gb = hcg.get_pipe_bwd_group() if hasattr(hcg, "get_pipe_bwd_group") else g
        self.group = g.group if g is not None else None
        self.group_bwd = gb.group if gb is not None else self.group
        self.ranks = g.ranks if g is not None else [0]
        self.stage = hcg.pp_rank
        self.nstages = hcg.pp_degree
        self._warm = False
        self._sends = []

    def warmup(self, device):
        """One collective over each pipe communicator before the first grouped
        p2p call: RCCL/NCCL require every rank of the group to take part in
        the call that creates the communicator."""
        if not self._warm and self.group is not None and self.nstages > 1:
            t = torch.zeros(1, device=device)
            dist.all_reduce(t, group=self.group)
            if self.group_bwd is not self.group:
                dist.all_reduce(t, group=self.group_bwd)
        self._warm = True

    def _peer(self, delta):
        return self.ranks[(self.stage + delta) % self.nstages]

    def _post(self, group, send, send_peer, recv, recv_peer):
        ops = []
        if send is not None:
            ops.append(dist.P2POp(dist.isend, send.contiguous(), send_peer, group))
        if recv is not None:
            ops.append(dist.P2POp(dist.irecv, recv, recv_peer, group))
        if not ops:
            return None
        works = dist.batch_isend_irecv(ops)
        if recv is None:
            self._sends.extend(works)
            return None
        if len(works) == len(ops):       # one Work per op (gloo): split them
            self._sends.extend(works[:-1])
            return _Recv(recv, works[-1:])
        # one Work for the whole group (coalesced RCCL/NCCL): the receive's
        # wait covers the send as well -- never wait a Work twice (gloo hangs)
        return _Recv(recv, works)

    def post(self, send_next=None, send_prev=None, recv_prev=None, recv_next=None):
        """Post a forward-direction group (send_next / recv_prev) and a
        backward-direction group (send_prev / recv_next); returns
        ``(recv_prev_handle, recv_next_handle)`` (``None`` where not asked)."""
        hp = self._post(self.group, send_next, self._peer(1), recv_prev, self._peer(-1))
        hn = self._post(self.group_bwd, send_prev, self._peer(-1), recv_next, self._peer(1))
        return hp, hn

    def exchange(self, send_next=None, send_prev=None, recv_prev=None, recv_next=None):
        """Blocking form of :meth:`post` (receives complete on return)."""
        hp, hn = self.post(send_next, send_prev, recv_prev, recv_next)
        return (hp.wait() if hp is not None else None), (hn.wait() if hn is not None else None)

    def drain(self):
        """Retire every pending send (end of a schedule)."""
        for w in self._sends:
            w.wait()
        self._sends = []


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
        """Warm-up forwards, steady 1F1B, cool-down backwards.  The receive of
        the next forward input rides with the current activation send, and the
        receive of the next output gradient with the current input-gradient
        send, so both transfers run under the compute that follows; the
        compute stream waits for a receive only when it consumes it."""
        p2p = self.p2p
        first, last = p2p.stage == 0, p2p.stage == p2p.nstages - 1
        warmup = min(p2p.nstages - p2p.stage - 1, m)
        remaining = m - warmup
        ins, outs, losses = [], [], []
        n_bwd = [0]
        x_q, dy_q = [], []          # posted receives (forward inputs / output grads)
        n_x, n_dy = [0], [0]        # receives posted so far

        def want_x():
            return not first and n_x[0] < m

        def want_dy():
            return not last and n_dy[0] < m

        def post(send_next=None, send_prev=None, rx=False, rdy=False):
            bp = self._buf() if rx and want_x() else None
            bn = self._buf() if rdy and want_dy() else None
            hp, hn = p2p.post(send_next=send_next, send_prev=send_prev, recv_prev=bp,
                              recv_next=bn)
            if hp is not None:
                x_q.append(hp)
                n_x[0] += 1
            if hn is not None:
                dy_q.append(hn)
                n_dy[0] += 1

        def fwd(k):
            x = x_q.pop(0).wait() if not first else None
            if x is not None:
                x.requires_grad_(True)
            y = stage_fn(0, k, x)
            if last:
                losses.append(y.detach())
            ins.append(x)
            outs.append(y)
            return y

        def bwd():
            n_bwd[0] += 1
            if n_bwd[0] == m and on_last_backward is not None:
                on_last_backward()
            x, y = ins.pop(0), outs.pop(0)
            if last:
                y.backward()
            else:
                torch.autograd.backward(y, dy_q.pop(0).wait())
            return x.grad if x is not None else None

        post(rx=True)                                   # input of micro-batch 0
        for k in range(warmup):
            y = fwd(k)
            post(send_next=None if last else y.detach(), rx=True,
                 rdy=(k == warmup - 1))                 # first output grad
        if warmup == 0:
            post(rdy=True)
        for k in range(remaining):
            y = fwd(warmup + k)
            post(send_next=None if last else y.detach(), rx=True)
            dx = bwd()
            post(send_prev=None if first else dx, rdy=True)
        for k in range(warmup):
            dx = bwd()
            post(send_prev=None if first else dx, rdy=True)
        p2p.drain()
        assert not x_q and not dy_q, "pipeline receive queue not drained"
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
        of this rank together with the receives it needs next (one grouped call
        per direction), and the k-th send on a link always meets the k-th
        receive on the other side (the chunk shift on the ring edge is a +P
        unit shift, which preserves order), so the schedule cannot deadlock;
        receives are waited for where consumed.  Requires ``m % P == 0``.
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
                x = inputs[c].pop(0).wait()
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
                torch.autograd.backward(y, grads[c].pop(0).wait())
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
            hp, hn = p2p.post(send_next=send_next, send_prev=send_prev, recv_prev=bp,
                              recv_next=bn)
            if hp is not None:
                inputs[fchunk(recv_for_fwd)].append(hp)
            if hn is not None:
                grads[bchunk(recv_for_bwd)].append(hn)

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
        p2p.drain()
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
                p2p.post(send_next=y)
        p2p.drain()
        if last:
            return torch.stack(losses).sum()
        return None
