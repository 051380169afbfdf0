"""LSTM sequence predictor (reference LSTM-TensorFlow-IO-Kafka/cardata-v2.py).

Reference stack (cardata-v2.py:177-183, look_back = 1, batch_size = 1):

    LSTM(32, relu, return_sequences=True, input_shape=(look_back, 18))
    LSTM(16, relu)
    RepeatVector(look_back)
    LSTM(16, relu, return_sequences=True)
    LSTM(32, relu, return_sequences=True)
    TimeDistributed(Dense(18))
    compile(metrics=['accuracy'], loss='mean_squared_error', optimizer='adam')

18 642 parameters.  Task: given a window of ``look_back`` normalised events,
predict the next event (``dataset.skip(look_back)``, :199-206).  BASELINE config 3
uses the 2-layer variant ``LSTM(32, seq) -> LSTM(16) -> Dense(18)`` with
``seq_len = 50`` (:func:`LSTMPredictor.two_layer`).

Every LSTM layer runs as :func:`streamml.ops.lstm.lstm` (fused HIP recurrence on
ROCm); dense heads are bf16 GEMMs; all parameters live in one flat buffer so the
optimizer step is one HIP Adam launch and DP is one RCCL all-reduce.
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ckpt import h5 as ckh5
from ..nn import keras_config as kc
from ..nn.callbacks import Callback, History
from ..ops.adam import FlatAdam, FlatParams
from ..ops.dense import dense as dense_op
from ..ops.loss import mse_accuracy
from ..ops.lstm import lstm as lstm_op

# layer spec: ("lstm", units, return_sequences, activation) | ("repeat", n) | ("dense", units, time_distributed)
REFERENCE_STACK = [("lstm", 32, True, "relu"), ("lstm", 16, False, "relu"), ("repeat", None),
                   ("lstm", 16, True, "relu"), ("lstm", 32, True, "relu"), ("dense", 18, True)]
TWO_LAYER_STACK = [("lstm", 32, True, "relu"), ("lstm", 16, False, "relu"), ("dense", 18, False)]


def _orthogonal(rows: int, cols: int, rng: np.random.Generator) -> np.ndarray:
    a = rng.standard_normal((max(rows, cols), min(rows, cols)))
    q, r = np.linalg.qr(a)
    q = q * np.sign(np.diag(r))
    return (q if rows >= cols else q.T)[:rows, :cols].astype(np.float32)


def _glorot(fi: int, fo: int, rng) -> np.ndarray:
    lim = math.sqrt(6.0 / (fi + fo))
    return rng.uniform(-lim, lim, size=(fi, fo)).astype(np.float32)


_FOLD = os.environ.get("SML_LSTM_FOLD", "1") != "0"


def _fwd2() -> bool:
    """SML_LSTM_FWD2=0: two single-layer forward launches instead of the stacked one (A/B;
    read per step)."""
    return os.environ.get("SML_LSTM_FWD2", "1") != "0"


def _headfuse() -> bool:
    """SML_LSTM_HEADFUSE=0: the Dense head as six per-kernel launches (K1 forward, mse_acc + fold, K2
    weight gradient + slab sum, K1 for dh) instead of the fused head (lstm_head.hip: one pass over the
    rows + one fold launch; A/B, read per step).  The per-kernel path rounds exactly as the autograd
    path does (tests/test_lstm_gpu.py test_fused_step_matches_autograd_step pins it); the fused
    head sums in another order."""
    return os.environ.get("SML_LSTM_HEADFUSE", "1") != "0"


def _slab2() -> bool:
    """SML_LSTM_SLAB2=0: each LSTM layer's weight-gradient slabs reduced right after its backward (two
    launches) instead of both in one launch before Adam (A/B; read per step)."""
    return os.environ.get("SML_LSTM_SLAB2", "1") != "0"


def _slab2adam() -> bool:
    """SML_LSTM_SLAB2ADAM=0: Adam as its own launch after the paired slab sum (A/B; read per step).
    Default: the paired slab sum applies Adam itself (dense.hip slab_sum2_kernel<ADAM>, bit-identical:
    sml_adam.h), one launch fewer per step."""
    return os.environ.get("SML_LSTM_SLAB2ADAM", "1") != "0"


def _frag() -> bool:
    """SML_LSTM_FRAG=0: the stacked two-layer step keeps h1 / h2 / dX as [B, T, U] rows instead of the
    fragment-native layout (A/B; read per step).  Fragment-native, every per-step h / dh / x access of
    a wave is one contiguous 512-byte piece per 16-sequence tile (lstm_fused.hip FR)."""
    return os.environ.get("SML_LSTM_FRAG", "1") != "0"


def _bwd2() -> bool:
    """SML_LSTM_BWD2=1: the bottom two layers' backward in ONE launch (lstm_fused_stack.hip)
    instead of two (read per step).  Off by default: correct (bit-identical to two launches
    up to fp32 summation order) but slower on MI355X -- one wave per SIMD carries both
    layers' dependency chains, 501 us vs 243 + 236 us for the two launches at the seq-50
    config, 88.8 vs 91.7 M windows/s (profiles/r05/lstm/ab_r05g_bwd2.txt)."""
    return os.environ.get("SML_LSTM_BWD2", "0") == "1"


class LSTMPredictor:
    def __init__(self, look_back: int = 1, features: int = 18, stack=None, device="auto", seed: int = 0,
                 name: str = "sequential", lr: float = 1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        if device in (None, "auto"):
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.look_back, self.features, self.name = int(look_back), int(features), name
        self.stack = [tuple(s) for s in (stack or REFERENCE_STACK)]
        self.hp = dict(lr=lr, beta_1=beta_1, beta_2=beta_2, epsilon=epsilon)
        rng = np.random.default_rng(seed)
        shapes, init, self.layers = [], [], []
        counts: Dict[str, int] = {}
        dim = self.features
        seq = True   # current tensor has a time axis
        for spec in self.stack:
            kind = spec[0]
            lname = kind if kind != "dense" or not spec[2] else "time_distributed"
            k = counts.get(lname, 0)
            counts[lname] = k + 1
            lname = lname if k == 0 else f"{lname}_{k}"
            if kind == "lstm":
                u = int(spec[1])
                if not seq:
                    raise ValueError("LSTM needs a sequence input (add a RepeatVector)")
                W, Uw, b = _glorot(dim, 4 * u, rng), _orthogonal(u, 4 * u, rng), np.zeros(4 * u, np.float32)
                b[u:2 * u] = 1.0   # unit_forget_bias
                self.layers.append(dict(kind="lstm", name=lname, units=u, return_sequences=bool(spec[2]),
                                        activation=spec[3], params=len(shapes), n=3, in_dim=dim))
                shapes += [(dim, 4 * u), (u, 4 * u), (4 * u,)]
                init += [W, Uw, b]
                dim, seq = u, bool(spec[2])
            elif kind == "repeat":
                n = int(spec[1] or self.look_back)
                self.layers.append(dict(kind="repeat", name=lname if k == 0 else lname, n=n))
                seq = True
            elif kind == "dense":
                u = int(spec[1])
                td = bool(spec[2])
                self.layers.append(dict(kind="dense", name=lname, units=u, td=td, params=len(shapes), n=2,
                                        in_dim=dim))
                shapes += [(dim, u), (u,)]
                init += [_glorot(dim, u, rng), np.zeros(u, np.float32)]
                dim = u
            else:
                raise ValueError(f"unknown layer kind {kind}")
        for L in self.layers:
            if L["kind"] == "repeat":
                L["name"] = "repeat_vector" if L["name"] == "repeat" else L["name"].replace("repeat", "repeat_vector")
        self.fp = FlatParams(shapes, self.device, init)
        self.opt = FlatAdam(self.fp, **self.hp)
        self._acc = np.zeros(4)   # loss*n, correct, n, batches
        self.stop_training = False
        self.last_fit_engine = None

    @classmethod
    def reference(cls, look_back: int = 1, **kw) -> "LSTMPredictor":
        return cls(look_back=look_back, stack=REFERENCE_STACK, **kw)

    @classmethod
    def two_layer(cls, look_back: int = 50, **kw) -> "LSTMPredictor":
        return cls(look_back=look_back, stack=TWO_LAYER_STACK, **kw)

    # ------------------------------------------------------------------ model
    def count_params(self) -> int:
        return int(self.fp.n)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        P = self.fp.params
        h = x
        for L in self.layers:
            if L["kind"] == "lstm":
                W, Uw, b = P[L["params"]:L["params"] + 3]
                h = lstm_op(h, W, Uw, b, L["activation"], return_sequences=L["return_sequences"])
            elif L["kind"] == "repeat":
                h = h.unsqueeze(1).expand(h.shape[0], L["n"], h.shape[-1]).contiguous()
            else:
                K, b = P[L["params"]:L["params"] + 2]
                h = dense_op(h, K, b)          # K1/K2 tall-skinny MFMA kernels on ROCm
        return h

    def _loss(self, y_pred: torch.Tensor, y: torch.Tensor):
        """Keras MSE (an (n, F) target broadcasts over (n, T, F) output steps) + accuracy count:
        one fused HIP kernel on ROCm (K3 + K6), torch ops on CPU."""
        return mse_accuracy(y_pred, y)

    def train_step(self, x: torch.Tensor, y: torch.Tensor, global_batch: Optional[int] = None, allreduce=None):
        n = x.shape[0]
        plan = self._fused_plan()
        if (plan is not None and isinstance(x, torch.Tensor) and isinstance(y, torch.Tensor) and x.is_cuda
                and x.dim() == 3 and y.dim() == 2 and n > 0):
            return self._fused_step(plan, x, y, global_batch, allreduce)
        self.fp.zero_grad()
        y_pred = self.forward(x)
        loss, correct = self._loss(y_pred, y)
        scale = n / float(global_batch or n)   # mean over the global batch under DP
        (loss * scale).backward()
        self.opt.step(allreduce=allreduce)
        return loss.detach(), correct.detach()

    def _fused_plan(self):
        """Whether a train step can run as explicit kernel calls (no autograd graph), and how.

        Two stack shapes qualify:
          * fused LSTM layers (the last one ``return_sequences=False``) and one Dense head --
            :meth:`two_layer`;
          * an encoder of fused LSTM layers ending in ``return_sequences=False``, a
            RepeatVector, a decoder of ``return_sequences=True`` LSTM layers and a
            TimeDistributed Dense head -- the reference stack (:meth:`reference`,
            LSTM-TensorFlow-IO-Kafka/cardata-v2.py:172-209).
        Builds, once, the int32 maps that scatter each layer's weight-gradient slab straight
        into the flat gradient buffer."""
        if getattr(self, "_plan_built", False):
            return self._plan
        self._plan_built, self._plan = True, None
        if self.device.type != "cuda":
            return None
        from ..ops.dense import supported as dense_ok
        from ..ops.loss import supported as mse_ok
        from ..ops.lstm import fused_supported
        body, head = self.layers[:-1], self.layers[-1]
        if not body or head["kind"] != "dense" or not mse_ok(head["units"]) or not dense_ok(head["in_dim"], head["units"]):
            return None
        kinds = [L["kind"] for L in body]
        if kinds.count("repeat") > 1 or any(k not in ("lstm", "repeat") for k in kinds):
            return None
        if "repeat" in kinds:
            r = kinds.index("repeat")
            pre, post, repeat = body[:r], body[r + 1:], body[r]["n"]
            if not pre or not post or not head["td"]:
                return None
            if any(L["return_sequences"] for L in pre[-1:]) or any(not L["return_sequences"] for L in post):
                return None
        else:
            pre, post, repeat = body, [], None
            if head["td"]:
                return None
        if any(L["return_sequences"] != (i < len(pre) - 1) for i, L in enumerate(pre)):
            return None
        if any(not fused_supported(L["units"], L["in_dim"]) for L in pre + post):
            return None
        from ..ops._ext import load_c
        C = load_c()
        off = self.fp.offsets
        maps = []
        for L in pre + post:
            u, IN = L["units"], L["in_dim"]
            G4, ldw = 4 * u, C.lstm_fused_dx_ld(IN)
            S = C.lstm_fused_slab(u, IN)
            mp = np.full(S, -1, np.int64)
            oW, oU, ob = (int(off[L["params"] + k]) for k in range(3))
            m, f = np.meshgrid(np.arange(G4), np.arange(ldw), indexing="ij")   # slab [G4][ldw] = dW^T
            mp[:G4 * ldw] = np.where(f < IN, oW + f * G4 + m, -1).ravel()
            m, uu = np.meshgrid(np.arange(G4), np.arange(u), indexing="ij")   # [G4][u] = dU^T
            mp[G4 * ldw:G4 * (ldw + u)] = (oU + uu * G4 + m).ravel()
            mp[G4 * (ldw + u):] = ob + np.arange(G4)
            assert G4 * (ldw + u + 1) == S
            maps.append(torch.as_tensor(mp.astype(np.int32), device=self.device))
        K, N = head["in_dim"], head["units"]
        KP, NP = 16 * C.dense_tiles(K), 16 * C.dense_tiles(N)
        S = C.dense_wgrad_slab(K, N)
        mp = np.full(S, -1, np.int64)
        oK, ob = int(off[head["params"]]), int(off[head["params"] + 1])
        k, nn = np.meshgrid(np.arange(KP), np.arange(NP), indexing="ij")
        mp[:KP * NP] = np.where((k < K) & (nn < N), oK + k * N + nn, -1).ravel()
        mp[KP * NP:KP * NP + NP] = np.where(np.arange(NP) < N, ob + np.arange(NP), -1)
        head_map = torch.as_tensor(mp.astype(np.int32), device=self.device)
        for m_ in maps + [head_map]:   # the kernels scatter through these unchecked
            assert int(m_.max()) < self.fp.n_pad and int(m_.min()) >= -1
        # the flat slots no LSTM slab map covers (the head's, the padding): updated from the gradient
        # as it stands when the paired slab sum applies Adam itself
        covered = np.concatenate([m_.cpu().numpy() for m_ in maps])
        rest = np.setdiff1d(np.arange(self.fp.n_pad), covered[covered >= 0]).astype(np.int32)
        assert rest.size == 0 or (int(rest.min()) >= 0 and int(rest.max()) < self.fp.n_pad)   # scattered unchecked
        self._plan = dict(pre=pre, post=post, repeat=repeat, head=head, maps=maps, head_map=head_map,
                          acc=torch.zeros(2, device=self.device), rest=torch.as_tensor(rest, device=self.device))
        return self._plan

    def _fused_step(self, plan, x, y, global_batch, allreduce):
        """One train step as explicit kernel calls on the flat buffers: per LSTM layer one
        fused forward and one fused backward (weight-gradient slabs reduced straight into
        the flat gradient through ``plan['maps']``), RepeatVector as a broadcast copy of
        h_T (its backward: the sum over the repeated steps), the Dense / TimeDistributed
        head on K1/K2, the fused MSE + accuracy kernel (target broadcast over the
        repeated steps), one Adam launch (+ one flat-gradient all-reduce under DP).  Same
        kernels and rounding points as the autograd path, ~20 fewer small launches per step."""
        from ..ops._ext import load_c
        from ..ops.lstm import ACT
        C = load_c()
        P, grad = self.fp.params, self.fp.grad
        n = x.shape[0]
        if not (x.stride(2) == 1 and x.stride(1) == x.shape[2] and x.stride(0) >= 0):
            x = x.contiguous()
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        pre, post, R = plan["pre"], plan["post"], plan["repeat"]
        saved = []
        h = x
        stack = pre + post
        first = 0
        frag = False   # layers 1 and 2 exchange fragment-native sequences (only h_T leaves the pair)
        hlast = None
        if _fwd2() and len(pre) >= 2 and x.dtype == torch.float32:
            # the first two layers (U 32 -> 16) in ONE forward launch: layer 1's h feeds layer 2
            # from registers (lstm_fused_fwd.hip fwd2); the same saved h / c as two launches
            L1, L2 = pre[0], pre[1]
            W1, U1, b1 = (t.detach() for t in P[L1["params"]:L1["params"] + 3])
            W2, U2, b2 = (t.detach() for t in P[L2["params"]:L2["params"] + 3])
            a1, a2 = ACT[L1["activation"]], ACT[L2["activation"]]
            if C.lstm_fused_fwd2_supported(x.shape[2], U1.shape[0], U2.shape[0], a1, a2):
                frag = (_frag() and not _bwd2() and len(pre) == 2 and not post
                        and C.lstm_fused_frag_supported(U1.shape[0], x.shape[2], False, False)
                        and C.lstm_fused_frag_supported(U2.shape[0], U1.shape[0], True, True))
                hs1, c1, hs2, c2, hlast = C.lstm_fused_fwd2(x, W1, U1, b1, W2, U2, b2, a1, a2, frag)
                saved += [(x, hs1, c1), (hs1, hs2, c2)]
                h, first = hs2, 2
        for L in stack[first:]:
            if L is (post[0] if post else None):   # RepeatVector: h_T broadcast over R steps
                # fp32 (exact widening of the bf16 h_T), as the autograd path feeds it: the
                # decoder's dx then comes back fp32 and is summed before one bf16 rounding
                h = h[:, -1].float().unsqueeze(1).expand(n, R, h.shape[-1]).contiguous()
            W, Uw, b = P[L["params"]:L["params"] + 3]
            hs, c = C.lstm_fused_fwd(h, W.detach(), Uw.detach(), b.detach(), None, None, ACT[L["activation"]])
            saved.append((h, hs, c))
            h = hs
        hd = plan["head"]
        K, bh = (t.detach() for t in P[hd["params"]:hd["params"] + 2])
        hin = h.reshape(n * R, h.shape[-1]) if R else (hlast if frag else h[:, -1])   # bf16, in place when h_T
        yt = y.to(device=self.device, dtype=torch.float32).contiguous()
        acc = plan["acc"]
        scale = n / float(global_batch or n)           # mean over the global batch under DP
        # this step's (loss, accuracy) and the Adam step count come out of the loss kernel's fold
        # launch (SML_LSTM_FOLD=0: a division, a copy and a counter add on the stream instead)
        fold = _FOLD
        metrics = torch.empty(2, device=self.device) if fold else None
        n_out = hin.shape[0] * K.shape[1]
        if not R and _headfuse() and K.shape[0] == 16 and K.shape[1] <= 32:
            # the Dense head in one pass (lstm_head.hip): forward, MSE + accuracy, dW / db into the flat
            # gradient, dh = dy . K^T -- 2 launches where the per-kernel path below takes 6
            dh = C.lstm_head(hin, K, bh, yt, 2.0 / n_out * scale, grad, plan["head_map"], acc, out=metrics,
                             div0=float(n_out), div1=1.0, counter=self.fp.iter if fold else None)
        else:
            y_pred = C.dense_fwd(hin, K, bh, 0, False, 1024, False)
            dy = torch.empty_like(y_pred)
            C.mse_acc(y_pred, yt, R or 1, 2.0 / n_out * scale, dy, acc, reset=True,   # acc = this step's sums
                      out=metrics, div0=float(n_out), div1=float(R or 1), counter=self.fp.iter if fold else None)
            C.dense_wgrad(hin, dy, 0, True, 1024, grad, plan["head_map"])
            dh = C.dense_fwd(dy, K, None, 0, True, 1024, True)   # dh = dy . K^T, bf16
        layers = pre + post
        # two LSTM layers: both weight-gradient slab sums in ONE launch after the second backward
        pair = len(layers) == 2 and not R and _slab2()
        deferred = []
        for i in range(len(layers) - 1, -1, -1):
            L = layers[i]
            xin, hs, c = saved[i]
            W, Uw, b = (t.detach() for t in P[L["params"]:L["params"] + 3])
            last_only = i == len(pre) - 1
            if R and i >= len(pre):
                dh = dh.view(n, R, -1)
            if i == 1 and not frag and _bwd2() and saved[0][0].dtype == torch.float32:
                # the bottom two layers' backward in ONE launch (lstm_fused_stack.hip): layer 2's
                # dX reaches layer 1 in registers, h1 is read once
                L0 = layers[0]
                W0, U0, b0 = (t.detach() for t in P[L0["params"]:L0["params"] + 3])
                x0, hs0, c0 = saved[0]
                a0, a1 = ACT[L0["activation"]], ACT[L["activation"]]
                if C.lstm_fused_bwd2_supported(x0.shape[2], U0.shape[0], Uw.shape[0], a0, a1) and \
                        dh.dim() == (2 if last_only else 3):
                    C.lstm_fused_bwd2(x0, hs0, c0, hs, c, dh, W0, U0, b0, W, Uw, b, a0, last_only, grad,
                                      plan["maps"][0], plan["maps"][1])
                    break
            out = C.lstm_fused_bwd(dh, c, hs, xin, None, None, W, Uw, b, ACT[L["activation"]], i > 0, False,
                                   last_only, grad, plan["maps"][i], frag and i < 2, defer_sum=pair)
            if pair:
                deferred.append((out[1], plan["maps"][i]))
            dh = out[0]
            if R and i == len(pre):   # RepeatVector backward: the repeated steps' gradients summed
                dh = (dh.view(n, -1) if R == 1 else dh.sum(1)).to(torch.bfloat16)
        if len(deferred) == 2 and allreduce is None and fold and self.opt.on_gpu and _slab2adam():
            # the step's last launch: both slab sums + Adam over every parameter (the step count was
            # advanced by the head's fold launch)
            o = self.opt
            C.slab_sum2(deferred[0][0], deferred[0][1], deferred[1][0], deferred[1][1], grad, params=self.fp.flat,
                        m=self.fp.m, v=self.fp.v, iter=self.fp.iter, lr=o.lr, beta1=o.b1, beta2=o.b2, eps=o.eps,
                        gscale=1.0, rest=plan["rest"])
        else:
            if len(deferred) == 2:
                C.slab_sum2(deferred[0][0], deferred[0][1], deferred[1][0], deferred[1][1], grad)
            self.opt.step(allreduce=allreduce, counted=fold)
        if fold:
            return metrics[0], metrics[1]   # acc is overwritten by the next step, metrics is this step's own
        # device-tensor divisors: an IEEE division, as the fold launch's (a Python-scalar divisor is a
        # reciprocal multiply in torch's kernel, which can differ in the last bit)
        div = torch.tensor([float(n_out), float(R or 1)], device=self.device)
        correct = acc[1] / div[1] if R else acc[1].clone()
        return acc[0] / div[0], correct

    # ------------------------------------------------------------------ training
    def fit(self, x, y=None, epochs: int = 1, batch_size: int = 1, verbose: int = 1, take: Optional[int] = None,
            callbacks: Optional[Sequence[Callback]] = None, shuffle: bool = False, normalize: bool = True,
            initial_epoch: int = 0, seed: int = 0, engine: str = "auto"):
        """``x``: windows [n, T, F] + ``y`` next rows [n, F], or a Stream (windows built here).

        ``engine``: ``"persistent"`` runs each epoch as ONE launch of the Keras-step kernel
        (``ops/lstm_persistent.py``; the reference stack at look_back 1, batch <= 32,
        one replica), ``"autograd"`` one fused-kernel train_step per batch, ``"auto"``
        the persistent kernel whenever it applies."""
        from ..data.stream import Stream
        from ..parallel.dp import allreduce_sum_
        import torch.distributed as dist

        pg = dist.is_available() and dist.is_initialized()
        world = dist.get_world_size() if pg else 1
        # any process group (also a 1-rank one, SML_FORCE_PG=1) takes the data-parallel path:
        # fused no-autograd steps + one flat-gradient RCCL all-reduce per step
        allreduce = allreduce_sum_ if pg else None
        hist = History()
        cbs = [hist] + list(callbacks or [])
        for cb in cbs:
            cb.set_model(self)
            cb.on_train_begin()
        if isinstance(x, Stream):
            st = x.normalize() if normalize else x
            if self.device.type == "cuda":
                # the event rows go to the device once; windows are strided views over them
                # (sliding_windows), read in place by the fused LSTM kernels
                from ..data.stream import sliding_windows
                rows = st.collect().x
                if world > 1 and x.shard is None:   # contiguous row shard per replica (+ the look_back overlap)
                    from ..parallel.dp import shard_range
                    nw = max(len(rows) - self.look_back, 0)
                    s0, s1 = shard_range(nw, dist.get_rank(), world)
                    rows = rows[s0:s1 + self.look_back]
                base = torch.as_tensor(np.ascontiguousarray(rows, np.float32), device=self.device)
                xd, yd = sliding_windows(base, self.look_back)
                world_sharded = True
            else:
                wins = [w for w in st.windows(self.look_back)]
                xs = np.concatenate([w[0] for w in wins]) if wins else np.zeros((0, self.look_back, self.features))
                ys = np.concatenate([w[1] for w in wins]) if wins else np.zeros((0, self.features))
                world_sharded = x.shard is not None   # kafka(shard=...): this rank's own partitions' windows
        elif isinstance(x, torch.Tensor) and x.device == self.device:
            # device tensors (e.g. data.stream.sliding_windows views) are used as they are
            xd = x if x.dtype == torch.float32 else x.float()
            yd = torch.as_tensor(y, device=self.device).float()
            if world > 1:
                from ..parallel.dp import shard_range
                s0, s1 = shard_range(len(xd), dist.get_rank(), world)
                xd, yd = xd[s0:s1], yd[s0:s1]
            world_sharded = True
        else:
            xs, ys = np.asarray(x, np.float32), np.asarray(y, np.float32)
            world_sharded = False
        device_input = (isinstance(x, Stream) and self.device.type == "cuda") or (
            isinstance(x, torch.Tensor) and x.device == self.device)
        if not device_input:
            if world > 1 and not world_sharded:   # contiguous shard per replica (as Autoencoder.fit)
                from ..parallel.dp import shard_range
                s0, s1 = shard_range(len(xs), dist.get_rank(), world)
                xs, ys = xs[s0:s1], ys[s0:s1]
            xd = torch.as_tensor(xs, dtype=torch.float32, device=self.device)
            yd = torch.as_tensor(ys, dtype=torch.float32, device=self.device)
        n = len(xd)
        nb = math.ceil(n / batch_size)
        ns = [n]
        if world > 1:
            # one all-reduce per step: every rank must run the same step count (shards may
            # differ by a few windows -- the rank with more drops its excess, as drop_last).
            # Every rank's row count, once: step b's global batch is the rows ALL ranks train in
            # it, so a short last batch averages over exactly those rows
            from ..parallel.dp import agree
            r_ = dist.get_rank()
            ns = agree([n if i == r_ else 0 for i in range(world)], None, ["sum"] * world)
            nb = min(math.ceil(v / batch_size) for v in ns)
        if take is not None:
            nb = min(nb, take)
        from ..ops import lstm_persistent as lp
        persistent = engine == "persistent" or (
            engine == "auto" and not pg and lp.supported(self) and batch_size <= lp.MAX_BATCH and n > 0)
        if persistent:
            if not (lp.supported(self) and not pg and batch_size <= lp.MAX_BATCH):
                raise ValueError("engine='persistent' needs the reference stack at look_back 1, batch <= "
                                 f"{lp.MAX_BATCH}, one replica")
            if not lp.check_inactive(self):
                raise RuntimeError("recurrent / forget-gate Adam moments are non-zero: the look_back-1 kernel "
                                   "would not reproduce their Keras updates (use engine='autograd')")
            self.last_fit_engine = "persistent"
            return self._fit_persistent(xd, yd, n, nb, epochs, batch_size, verbose, cbs, hist, shuffle, seed,
                                        initial_epoch)
        plan = self._fused_plan()
        self.last_fit_engine = ("fused" if plan is not None else "autograd") + ("+allreduce" if pg else "")
        from ..parallel.fault import maybe_inject
        rank = dist.get_rank() if world > 1 else 0
        gstep = 0
        for epoch in range(initial_epoch, epochs):
            t0 = time.perf_counter()
            tot_loss = torch.zeros((), device=self.device)
            tot_corr = torch.zeros((), device=self.device)
            rows = 0
            order = None
            if shuffle:   # epoch-keyed permutation: resumable
                order = torch.as_tensor(np.random.default_rng([seed, rank, epoch]).permutation(n), device=self.device)
            for b in range(nb):
                sl = slice(b * batch_size, (b + 1) * batch_size)
                xb = xd[order[sl]] if order is not None else xd[sl]
                yb = yd[order[sl]] if order is not None else yd[sl]
                maybe_inject(gstep, rank)
                gb = sum(min(batch_size, max(0, v - b * batch_size)) for v in ns) if world > 1 else len(xb)
                loss, corr = self.train_step(xb, yb, global_batch=gb, allreduce=allreduce)
                gstep += 1
                tot_loss += loss * len(xb)
                tot_corr += corr
                rows += len(xb)
            logs = {"loss": float(tot_loss) / max(rows, 1), "accuracy": float(tot_corr) / max(rows, 1),
                    "_seconds": time.perf_counter() - t0, "_rows": rows}
            if verbose:
                print(f"Epoch {epoch + 1}/{epochs} - {nb} steps - loss: {logs['loss']:.4f} - "
                      f"accuracy: {logs['accuracy']:.4f}", flush=True)
            for cb in cbs:
                cb.on_epoch_end(epoch, logs)
            if self.stop_training:
                break
        for cb in cbs:
            cb.on_train_end()
        return hist

    def _fit_persistent(self, xd, yd, n, nb, epochs, batch_size, verbose, cbs, hist, shuffle, seed, initial_epoch):
        from ..ops import lstm_persistent as lp
        for epoch in range(initial_epoch, epochs):
            t0 = time.perf_counter()
            order = None
            if shuffle:
                order = torch.as_tensor(np.random.default_rng([seed, 0, epoch]).permutation(n).astype(np.int32),
                                        device=self.device)
            out = lp.train_steps(self, xd, yd, batch_size, nb, 0, order)
            rows = min(n, nb * batch_size)
            sizes = torch.full((nb,), float(batch_size), device=self.device)
            sizes[-1] = float(rows - (nb - 1) * batch_size)
            tot = torch.stack([(out[:, 0] * sizes).sum(), out[:, 1].sum()]).cpu()
            logs = {"loss": float(tot[0]) / max(rows, 1), "accuracy": float(tot[1]) / max(rows, 1),
                    "_seconds": time.perf_counter() - t0, "_rows": rows}
            if verbose:
                print(f"Epoch {epoch + 1}/{epochs} - {nb} steps - loss: {logs['loss']:.4f} - "
                      f"accuracy: {logs['accuracy']:.4f}", flush=True)
            for cb in cbs:
                cb.on_epoch_end(epoch, logs)
            if self.stop_training:
                break
        for cb in cbs:
            cb.on_train_end()
        return hist

    @torch.no_grad()
    def predict(self, x, batch_size: int = 1024, callbacks: Optional[Sequence[Callback]] = None):
        """Forecasts of windows ``x`` [n, look_back, features].

        A torch tensor already on the model's device stays there: batches are views of it and
        the result is a device tensor (no host round trip).  Host input is copied to the
        device once and the result comes back once, as numpy (Keras' return type).  Output
        callbacks get each batch's last-step forecasts as numpy."""
        on_dev = isinstance(x, torch.Tensor) and x.device == self.device
        xs = x if on_dev else torch.as_tensor(np.asarray(x, np.float32), device=self.device)
        outs = []
        for bi, s in enumerate(range(0, len(xs), batch_size)):
            out = self.forward(xs[s:s + batch_size])
            outs.append(out)
            for cb in callbacks or []:
                cb.set_model(self)
                o = out.detach().float().cpu().numpy()
                cb.on_predict_batch_end(bi, {"outputs": o.reshape(len(o), -1, self.features)[:, -1]})
        for cb in callbacks or []:
            cb.on_predict_end()
        if not outs:
            return torch.zeros((0,), device=self.device) if on_dev else np.zeros((0,), np.float32)
        res = torch.cat(outs) if len(outs) > 1 else outs[0]
        return res if on_dev else res.detach().cpu().numpy()

    # ------------------------------------------------------------------ persistence
    def weight_names(self) -> List[Tuple[str, List[str]]]:
        out = []
        for L in self.layers:
            if L["kind"] == "lstm":
                out.append((L["name"], [f"{L['name']}/kernel:0", f"{L['name']}/recurrent_kernel:0",
                                        f"{L['name']}/bias:0"]))
            elif L["kind"] == "dense":
                out.append((L["name"], [f"{L['name']}/kernel:0", f"{L['name']}/bias:0"]))
            else:
                out.append((L["name"], []))
        return out

    def model_config(self) -> dict:
        layers = []
        first = True
        for L in self.layers:
            if L["kind"] == "lstm":
                cfg = kc.lstm_config(L["name"], L["units"], L["activation"], L["return_sequences"],
                                     [None, self.look_back, self.features] if first else None)
                layers.append({"class_name": "LSTM", "config": cfg})
            elif L["kind"] == "repeat":
                layers.append({"class_name": "RepeatVector", "config": {"name": L["name"], "trainable": True,
                                                                        "dtype": "float32", "n": L["n"]}})
            else:
                d = kc.dense_config(L["name"] if not L["td"] else "dense", L["units"], "linear")
                if L["td"]:
                    layers.append({"class_name": "TimeDistributed", "config": {
                        "name": L["name"], "trainable": True, "dtype": "float32",
                        "layer": {"class_name": "Dense", "config": d}}})
                else:
                    layers.append({"class_name": "Dense", "config": d})
            first = False
        return kc.sequential(self.name, layers)

    def save(self, path: str, include_optimizer: bool = True) -> None:
        arrays = self.fp.get()
        layers, k = [], 0
        flat_names = []
        for lname, wnames in self.weight_names():
            ws = []
            for wn in wnames:
                ws.append((wn, arrays[k]))
                flat_names.append(wn)
                k += 1
            layers.append((lname, ws))
        opt = None
        if include_optimizer:
            it, m, v = self.opt.state()
            opt = list(zip(ckh5.adam_weight_names(flat_names), [np.array(it, np.int64)] + m + v))
        ckh5.save_keras_h5(path, self.model_config(), layers,
                           kc.training_config(self.hp["lr"], self.hp["beta_1"], self.hp["beta_2"],
                                              self.hp["epsilon"]), opt)

    @classmethod
    def load(cls, path: str, device="auto") -> "LSTMPredictor":
        ck = ckh5.load_keras_h5(path)
        cfg = ck.model_config["config"]
        stack, look_back, features = [], 1, 18
        for i, lyr in enumerate(cfg["layers"]):
            c = lyr["config"]
            if lyr["class_name"] == "LSTM":
                if "batch_input_shape" in c:
                    look_back, features = int(c["batch_input_shape"][1]), int(c["batch_input_shape"][2])
                stack.append(("lstm", int(c["units"]), bool(c["return_sequences"]), c["activation"]))
            elif lyr["class_name"] == "RepeatVector":
                stack.append(("repeat", int(c["n"])))
            elif lyr["class_name"] == "TimeDistributed":
                stack.append(("dense", int(c["layer"]["config"]["units"]), True))
            elif lyr["class_name"] == "Dense":
                stack.append(("dense", int(c["units"]), False))
            else:
                raise ValueError(f"unsupported layer {lyr['class_name']}")
        m = cls(look_back=look_back, features=features, stack=stack, device=device, name=cfg.get("name", "sequential"),
                **kc.optimizer_hparams(ck.training_config))
        m.fp.set(ck.flat_weights())
        if ck.optimizer_weights and len(ck.optimizer_weights) == 1 + 2 * len(m.fp.shapes):
            arr = [a for _, a in ck.optimizer_weights]
            k = len(m.fp.shapes)
            m.opt.load_state(int(np.asarray(arr[0]).reshape(-1)[0]), arr[1:1 + k], arr[1 + k:])
        return m
