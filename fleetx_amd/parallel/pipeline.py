"""Pipeline parallelism: 1F1B and interleaved (virtual-stage) schedules.

Capability parity: Paddle ``PipelineLayer`` / ``PipelineParallel.train_batch``
/ ``PipelineParallelWithInterleave`` reached from reference
``eager_engine.py:400-410,521,577`` and ``hybrid_model.py:862-962`` (P05,
N10-N12): the local batch is split into ``accumulate_steps`` micro-batches;
warm-up forwards, steady 1F1B, cool-down backwards; activations / grads of
``[micro_b, s, h]`` move between neighbouring stages; the last stage computes
the loss (averaged over micro-batches) and the tied embedding grad is reduced
between the first and last stage.

MI355X / RCCL design:
* every exchange is ONE grouped ``batch_isend_irecv`` (``ncclGroupStart/End``)
  on the pipe communicator.  RCCL runs the groups of one communicator in
  order on one stream and a group finishes only when all of its sends and
  receives have met their peers, so the posting order is what decides
  whether a schedule can deadlock.  The schedules therefore post
  MIRROR-IMAGE groups on both ends of every link, in the same order:
  ``{send y_k -> s+1, recv dy_j <- s+1}`` on stage s meets
  ``{send dx_j -> s, recv x_k+1 <- s}`` on stage s+1 (the steady-state
  pairing of Megatron-LM's 1F1B).  ``tests/test_pipeline_order_cpu.py``
  replays the posted groups of every schedule (1F1B, interleaved, forward-only,
  interleaved forward-only; P up to 8) against an in-order-per-communicator
  matcher (``parallel/p2p_replay.py``) and against host-blocking matching;
* with ``Distributed.comm.pp_split_directions`` activations and gradients
  get a communicator each (two groups per exchange); the same replay covers
  that mode;
* nothing waits for a SEND: the compute stream waits for a receive only where
  the received tensor is consumed (``_Recv.wait``; with RCCL a ``Work.wait``
  is a stream-level wait, not a host block).  Pending sends are retired at the
  end of the step;
* shapes are static (``[micro_b, s, h]`` in the model dtype), so there is no
  per-step shape handshake; ``Distributed.debug: fingerprint`` checks them
  (and the per-link order) pairwise over gloo (``collective_check.check_p2p``);
* gradient-bucket reductions of the flat grad buffer are armed only for the
  LAST backward of the step and overlap the cool-down phase.
"""
import torch
import torch.distributed as dist

from . import collective_check


class _GlooStaged:
    """A gloo p2p op on a DEVICE tensor, staged through host memory.  gloo
    moves the bytes from its own thread with no order against the GPU
    stream: a send could read an activation its producing kernel has not
    finished writing (the multi-rank rehearsal of ``bench.py`` over gloo saw
    NaN losses come and go with kernel timing).  The send copies to the host
    first (after the producer, on the current stream); the receive lands in a
    host buffer and is copied to the device tensor when waited."""

    __slots__ = ("work", "host", "dev")

    def __init__(self, work, host=None, dev=None):
        self.work, self.host, self.dev = work, host, dev

    def wait(self):
        self.work.wait()
        if self.dev is not None:
            self.dev.copy_(self.host, non_blocking=False)
            self.dev = None
        return True


def issue_dist(group, ops):
    """Issue ``ops`` (``[(kind, tensor, peer)]``, kind ``"send"``/``"recv"``,
    peer a global rank) as one grouped call; returns the ``Work`` list (one
    per op on gloo, one for the whole group on RCCL)."""
    if ops and ops[0][1].is_cuda and dist.get_backend(group) == "gloo":
        works = []
        for k, t, peer in ops:
            if k == "send":
                host = t.to("cpu")  # (synchronous: after the kernels that produce t)
                works.append(_GlooStaged(dist.isend(host, peer, group=group), host))
            else:
                host = torch.empty(t.shape, dtype=t.dtype)
                works.append(_GlooStaged(dist.irecv(host, peer, group=group), host, t))
        return works
    return dist.batch_isend_irecv([dist.P2POp(dist.isend if k == "send" else dist.irecv,
                                              t, peer, group) for k, t, peer in ops])


class _Recv:
    """A posted receive: ``wait()`` orders the consumer after the transfer and
    returns the buffer.  Receives of one coalesced group share the ``works``
    list, which is emptied by the first wait (never wait a Work twice)."""

    __slots__ = ("buf", "works")

    def __init__(self, buf, works):
        self.buf, self.works = buf, works

    def wait(self):
        for w in self.works:
            w.wait()
        self.works.clear()
        return self.buf


class P2P:
    def __init__(self, hcg, issue=None):
        self.hcg = hcg
        g = hcg.get_pipe_parallel_group()
        gb = hcg.get_pipe_bwd_group() if hasattr(hcg, "get_pipe_bwd_group") else g
        self.group = g.group if g is not None else None
        self.group_bwd = gb.group if gb is not None else self.group
        self.ranks = g.ranks if g is not None else [0]
        self.stage = hcg.pp_rank
        self.nstages = hcg.pp_degree
        self.issue = issue or issue_dist
        self._warm = issue is not None
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

    def _issue(self, group, ops):
        """One grouped call; returns ``{recv buffer id: _Recv}``."""
        if collective_check.enabled():
            collective_check.check_p2p(group, ops)
        works = list(self.issue(group, ops))
        handles = {}
        if len(works) == len(ops):          # one Work per op (gloo)
            for (kind, t, _), w in zip(ops, works):
                if kind == "recv":
                    handles[id(t)] = _Recv(t, [w])
                else:
                    self._sends.append(w)
            return handles
        # one Work for the whole group (coalesced RCCL): the receives' wait
        # covers the sends as well
        recvs = [t for kind, t, _ in ops if kind == "recv"]
        if not recvs:
            self._sends.extend(works)
        for t in recvs:
            handles[id(t)] = _Recv(t, works)
        return handles

    def post(self, send_next=None, send_prev=None, recv_prev=None, recv_next=None):
        """Post one exchange with the neighbouring stages; returns
        ``(recv_prev_handle, recv_next_handle)`` (``None`` where not asked).

        One communicator: all ops form ONE group.  Split directions: the
        activation-direction ops (send_next / recv_prev) and the
        gradient-direction ops (send_prev / recv_next) form one group each on
        their own communicator."""
        fwd, bwd = [], []
        if send_next is not None:
            fwd.append(("send", send_next.contiguous(), self._peer(1)))
        if recv_prev is not None:
            fwd.append(("recv", recv_prev, self._peer(-1)))
        if send_prev is not None:
            bwd.append(("send", send_prev.contiguous(), self._peer(-1)))
        if recv_next is not None:
            bwd.append(("recv", recv_next, self._peer(1)))
        if self.group_bwd is self.group:
            groups = [(self.group, fwd + bwd)]
        else:
            groups = [(self.group, fwd), (self.group_bwd, bwd)]
        handles = {}
        for g, ops in groups:
            if ops:
                handles.update(self._issue(g, ops))
        hp = handles.get(id(recv_prev)) if recv_prev is not None else None
        hn = handles.get(id(recv_next)) if recv_next is not None else None
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
    ``p2p`` injects a transport (the order replay of ``p2p_replay.py``).
    """

    def __init__(self, hcg, act_shape_fn, dtype, device, num_chunks=1, p2p=None):
        self.p2p = p2p if p2p is not None else P2P(hcg)
        self.hcg = hcg
        self.act_shape_fn = act_shape_fn
        self.dtype, self.device = dtype, device
        self.num_chunks = num_chunks
        self.p2p.warmup(device)

    def _buf(self):
        return torch.empty(self.act_shape_fn(), dtype=self.dtype, device=self.device)

    # ------------------------------------------------------------------ 1F1B
    def train_1f1b(self, m, stage_fn, on_last_backward=None):
        """Warm-up forwards, steady 1F1B, cool-down backwards (stage s runs
        ``min(P - s - 1, m)`` warm-up forwards).

        Posting order (mirror image on the two ends of every link):
        * warm-up: ``{recv x_i}``, forward, ``{send y_i}``;
        * before the steady phase: ``{recv x_w}``;
        * steady: forward k, ``{send y_k, recv dy_j}``, backward j,
          ``{send dx_j, recv x_k+1}`` (the last one is ``{send dx_j}``);
        * cool-down: ``{recv dy_j}``, backward j, ``{send dx_j}``.
        The compute stream waits for a receive only where it consumes it."""
        p2p = self.p2p
        first, last = p2p.stage == 0, p2p.stage == p2p.nstages - 1
        warmup = min(p2p.nstages - p2p.stage - 1, m)
        remaining = m - warmup
        ins, outs, losses = [], [], []
        n_bwd = [0]

        def recv_x():
            return None if first else p2p.post(recv_prev=self._buf())[0]

        def fwd(k, hx):
            x = hx.wait() if hx is not None else None
            if x is not None:
                x.requires_grad_(True)
            y = stage_fn(0, k, x)
            if last:
                losses.append(y.detach())
            ins.append(x)
            outs.append(y)
            return y

        def bwd(hdy):
            n_bwd[0] += 1
            if n_bwd[0] == m and on_last_backward is not None:
                on_last_backward()
            x, y = ins.pop(0), outs.pop(0)
            if last:
                y.backward()
            else:
                torch.autograd.backward(y, hdy.wait())
            return x.grad if x is not None else None

        for i in range(warmup):                 # never on the last stage
            y = fwd(i, recv_x())
            p2p.post(send_next=y.detach())
        hx = recv_x() if remaining > 0 else None
        for i in range(remaining):
            y = fwd(warmup + i, hx)
            hdy = None if last else p2p.post(send_next=y.detach(), recv_next=self._buf())[1]
            dx = bwd(hdy)
            if i == remaining - 1:
                hx = None
                if not first:
                    p2p.post(send_prev=dx)
            elif not first:
                hx = p2p.post(send_prev=dx, recv_prev=self._buf())[0]
        for i in range(warmup):
            hdy = p2p.post(recv_next=self._buf())[1]
            dx = bwd(hdy)
            if not first:
                p2p.post(send_prev=dx)
        p2p.drain()
        assert not ins and not outs, "pipeline activations not consumed"
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
        of this rank together with the receives it needs next as ONE group
        (Megatron-LM's ``send_forward_backward_recv_forward_backward``); each
        rank posts the same number of exchanges and the k-th send on a link
        meets the k-th receive on the other side (the chunk shift on the ring
        edge is a +P unit shift, which preserves order).  Receives are waited
        for where consumed.  Requires ``m % P == 0``.
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

    @torch.no_grad()
    def forward_only_interleaved(self, m, stage_fn):
        """Evaluation through the virtual-stage ring: micro-batch by
        micro-batch, chunk by chunk (``{recv x}``, forward, ``{send y}``)."""
        p2p = self.p2p
        P, V, r = p2p.nstages, self.num_chunks, p2p.stage
        losses = []
        for k in range(m):
            for c in range(V):
                first_v, last_v = r == 0 and c == 0, r == P - 1 and c == V - 1
                x = None if first_v else p2p.exchange(recv_prev=self._buf())[0]
                y = stage_fn(c, k, x)
                if last_v:
                    losses.append(y.detach())
                else:
                    p2p.post(send_next=y)
        p2p.drain()
        if r == P - 1:
            return torch.stack(losses).sum()
        return None
