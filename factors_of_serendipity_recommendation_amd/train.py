"""BPR training drop-ins: utils.BPRLoss (code/utils.py:34-53) and
Procedure.BPR_train_original (code/Procedure.py:26-57).

Same semantics, with the epoch's samples drawn on the GPU (``sampling.sample_device``) and shuffled
and batched on the device -- nothing goes through the host.  Every minibatch runs the model's
``bpr_loss``: for the LightGCN module of this package that is the HIP propagation forward and, in
backward, the same K-layer propagation of the gradient (A^ is symmetric), then torch's Adam.
"""
from __future__ import annotations

import time
from typing import Optional

import torch

from . import _lib, sampling
from .graph import _stream_ptr, require_gpu


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam as BPRLoss uses it (code/utils.py:41: lr only; betas (0.9, 0.999), eps 1e-8,
    no weight decay, no amsgrad), one ``lgx_adam_step`` launch per parameter instead of torch's
    ~7 multi-tensor passes.  State keys match torch's (step, exp_avg, exp_avg_sq), so a
    state_dict round-trips.  GPU f32 parameters only -- there is no CPU path."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                require_gpu(p)
                if p.dtype != torch.float32 or not p.is_contiguous() or p.grad.is_sparse:
                    raise TypeError("lgx Adam takes dense contiguous float32 parameters")
                st = self.state[p]
                if not st:
                    # the step count lives on the device (torch's capturable-Adam form), so that a
                    # graph-captured training step replays with a live count
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                elif not st["step"].is_cuda:  # a state_dict saved by torch's (non-capturable) Adam
                    st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
                st["step"].add_(1)
                g = p.grad.contiguous()
                _lib.check(_lib.lib().lgx_adam_step_dev(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                                                        st["exp_avg_sq"].data_ptr(), p.numel(), float(group["lr"]),
                                                        float(b1), float(b2), float(group["eps"]),
                                                        st["step"].data_ptr(), _stream_ptr(p.device)),
                           "lgx_adam_step_dev")
                # the kernel wrote p through a raw pointer: bump its version counter so that
                # version-keyed caches (LightGCN's eval-mode propagation) see the update
                torch.autograd.graph.increment_version(p)
        return loss


class BPRLoss:
    """utils.BPRLoss: Adam on the model's parameters, loss = bpr + decay * reg."""

    def __init__(self, recmodel, config: dict):
        self.model = recmodel
        self.weight_decay = config["decay"]
        self.lr = config["lr"]
        self.opt = Adam(recmodel.parameters(), lr=self.lr)

    def stageOne(self, users, pos, neg) -> float:
        loss, reg_loss = self.model.bpr_loss(users, pos, neg)
        loss = loss + reg_loss * self.weight_decay
        self.opt.zero_grad()
        loss.backward()
        self.opt.step()
        return loss.detach()


class _CapturedStep:
    """One full BPR minibatch -- bpr_loss, its backward (the fused loss gradient and the K-layer
    propagation of it) and the Adam step -- captured once as a hipGraph (torch.cuda.CUDAGraph) and
    replayed per minibatch: one host call instead of ~20 launches, so the epoch runs at the GPU's
    pace whatever the host does (the eager loop issues 0.26 ms of launches per 0.31 ms minibatch).
    Inputs are copied into static index buffers; the loss comes back in a static tensor.

    A replay repeats the host values and device addresses frozen at capture: lr / betas / eps and
    the decay factor are kernel scalars, the parameters and the optimizer state tensors are captured
    by address.  ``key`` records them; a change (an lr schedule, ``opt.load_state_dict`` replacing
    the state tensors, a new decay) makes the next minibatch re-capture instead of replaying."""

    def __init__(self, loss_class, batch_size: int, device):
        self.bs = batch_size
        self.u = torch.zeros(batch_size, dtype=torch.long, device=device)
        self.p = torch.zeros(batch_size, dtype=torch.long, device=device)
        self.n = torch.zeros(batch_size, dtype=torch.long, device=device)
        self.graph = None
        self.loss = None
        self.failed = False
        self.key = None
        self.captures = 0

    @staticmethod
    def capture_key(loss_class):
        opt = loss_class.opt
        groups = []
        for g in opt.param_groups:
            params = []
            for prm in g["params"]:
                st = opt.state.get(prm, {})
                params.append((prm.data_ptr(), tuple(st[k].data_ptr() if torch.is_tensor(st.get(k)) else None
                                     for k in ("step", "exp_avg", "exp_avg_sq"))))
            groups.append((float(g["lr"]), tuple(g["betas"]), float(g["eps"]), tuple(params)))
        return id(opt), float(loss_class.weight_decay), tuple(groups)

    def run(self, loss_class, u, p, n):
        self.u.copy_(u)
        self.p.copy_(p)
        self.n.copy_(n)
        if self.graph is not None and self.capture_key(loss_class) != self.key:
            self.graph = None  # frozen scalars / addresses changed: capture again
        if self.graph is None:
            dev = self.u.device
            # warm-up = this minibatch's real step, eager on a side stream (allocates the gradients,
            # the optimizer state and the engine's scratch before capture), then the capture
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                out = loss_class.stageOne(self.u, self.p, self.n)
            torch.cuda.current_stream(dev).wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(graph):
                    self.loss = loss_class.stageOne(self.u, self.p, self.n)
            except RuntimeError as e:  # a model whose step cannot be captured: train eagerly
                import warnings
                warnings.warn(f"BPR step capture failed ({e}); training without the graph")
                self.failed = True
                return out
            self.graph = graph
            self.key = self.capture_key(loss_class)
            self.captures += 1
            return out
        self.graph.replay()
        return self.loss


def _graph_ok(recommend_model, device) -> bool:
    """Capture only this package's LightGCN without edge dropout (the dropout graph is rebuilt per
    minibatch on the host); LGX_TRAIN_EAGER=1 keeps the eager loop."""
    import os
    from .model import LightGCN
    return (os.environ.get("LGX_TRAIN_EAGER", "0") != "1" and torch.device(device).type == "cuda"
            and isinstance(recommend_model, LightGCN) and not recommend_model.config.get("dropout", 0))


def _positives(dataset, device):
    if not hasattr(dataset, "_lgx_pos_csr"):
        dataset._lgx_pos_csr = sampling._positives(dataset.allPos, device)
    return dataset._lgx_pos_csr


def BPR_train_original(dataset, recommend_model, loss_class: BPRLoss, epoch: int, neg_k: int = 1, w=None,
                       batch_size: int = 2048, device="cuda", graph: Optional[bool] = None) -> str:
    """Procedure.BPR_train_original: one epoch of BPR minibatches; returns the same summary string."""
    Recmodel = recommend_model
    Recmodel.train()
    t0 = time.perf_counter()
    pos = _positives(dataset, device)
    per = max(1, dataset.trainDataSize // max(1, dataset.n_users))
    S = sampling.sample_device(pos, dataset.m_items, per_user=per, neg_num=neg_k).long()
    t_sample = time.perf_counter() - t0
    perm = torch.randperm(S.shape[0], device=S.device)  # utils.shuffle
    users, posItems, negItems = S[perm, 0], S[perm, 1], S[perm, 2]
    total_batch = len(users) // batch_size + 1
    aver_loss = torch.zeros((), device=S.device)
    if graph is None:
        graph = _graph_ok(Recmodel, device)
    step = None
    if graph:
        step = getattr(loss_class, "_lgx_captured", None)
        if step is None or step.bs != batch_size:
            step = loss_class._lgx_captured = _CapturedStep(loss_class, batch_size, S.device)
    Recmodel._lgx_trusted_indices = True  # the sampler's rows are in range by construction
    try:
        for batch_i, i in enumerate(range(0, len(users), batch_size)):  # utils.minibatch
            u, p, n = users[i:i + batch_size], posItems[i:i + batch_size], negItems[i:i + batch_size]
            if step is not None and not step.failed and u.numel() == batch_size:
                cri = step.run(loss_class, u, p, n)
            else:
                cri = loss_class.stageOne(u, p, n)
            aver_loss += cri
            if w is not None:
                w.add_scalar("BPRLoss/BPR", float(cri), epoch * int(len(users) / batch_size) + batch_i)
    finally:
        Recmodel._lgx_trusted_indices = False
        if step is not None:
            # replays wrote the parameters without the host seeing it: bump their versions so that
            # version-keyed caches (LightGCN's eval-mode propagation) see the new weights
            with torch.no_grad():
                for prm in Recmodel.parameters():
                    torch.autograd.graph.increment_version(prm)
    aver_loss = float(aver_loss) / total_batch
    return f"loss{aver_loss:.3f}-|Sample:{t_sample:.2f}|"
