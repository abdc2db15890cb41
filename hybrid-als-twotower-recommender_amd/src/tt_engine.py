"""Device two-tower engine: the Keras model of src/two_tower_model.py:38-119
(graph, MSE, Adam, fit loop) held as device tensors and driven through the
hrec_tt_* / hrec_adam_* kernels.

Dense parameters live in ONE flat f32 buffer laid out exactly like the
gradient block of hrec_tt_forward_backward
    W2[(d+32)*d] | b2[d] | gamma_i[d] | beta_i[d] | gamma_u[d] | beta_u[d] | W1[32] | b1[16]
so one hrec_adam_dense launch updates them all. Embedding tables get Keras'
sparse Adam (whole-table slot decay): all four tables in one grouped call,
or (rows of whole 16-B vectors) its phased form with the sweep of the
untouched rows on a side stream beside the forward / backward.
"""
import math
import os

import numpy as np
import torch

from . import _hrec

TABLES = ("user_emb", "item_emb", "man_emb", "cat_emb")


def dense_layout(d):
    """name -> (offset, shape) inside the flat dense buffer."""
    dz = d + 32
    layout, off = {}, 0
    for name, shape in (("w2", (dz, d)), ("b2", (d,)), ("ln_item_gamma", (d,)), ("ln_item_beta", (d,)),
                        ("ln_user_gamma", (d,)), ("ln_user_beta", (d,)), ("w1", (2, 16)), ("b1", (16,))):
        layout[name] = (off, shape)
        off += int(np.prod(shape))
    return layout, off


def keras_init(num_users, num_items, num_man, num_cat, d, seed):
    """Keras 2.8 initialisers: Embedding uniform(-0.05, 0.05); Dense kernel
    glorot_uniform, bias zeros; LayerNormalization gamma 1, beta 0. (Keras'
    own RNG stream is not reproducible outside TF; this one is seeded.)"""
    rng = np.random.default_rng(seed)

    def uni(shape, lim):
        return rng.uniform(-lim, lim, size=shape).astype(np.float32)

    p = {
        "user_emb": uni((num_users, d), 0.05),
        "item_emb": uni((num_items, d), 0.05),
        "man_emb": uni((num_man, 8), 0.05),
        "cat_emb": uni((num_cat, 8), 0.05),
        "w1": uni((2, 16), math.sqrt(6.0 / (2 + 16))),
        "b1": np.zeros(16, np.float32),
        "w2": uni((d + 32, d), math.sqrt(6.0 / (d + 32 + d))),
        "b2": np.zeros(d, np.float32),
        "ln_user_gamma": np.ones(d, np.float32),
        "ln_user_beta": np.zeros(d, np.float32),
        "ln_item_gamma": np.ones(d, np.float32),
        "ln_item_beta": np.zeros(d, np.float32),
    }
    return p


class AdamConfig:
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.lr = np.float32(learning_rate)
        self.b1 = np.float32(beta_1)
        self.b2 = np.float32(beta_2)
        self.eps = np.float32(epsilon)

    def coefficients(self, iterations):
        """OptimizerV2 Adam._prepare_local for local_step = iterations + 1, f32."""
        t = np.float32(iterations + 1)
        with np.errstate(all="ignore"):
            b1p = np.float32(np.power(self.b1, t, dtype=np.float32))
            b2p = np.float32(np.power(self.b2, t, dtype=np.float32))
            one = np.float32(1.0)
            sparse_lr = np.float32(self.lr * np.float32(np.sqrt(np.float32(one - b2p)) / np.float32(one - b1p)))
            dense_alpha = np.float32(np.float32(self.lr * np.sqrt(np.float32(one - b2p))) / np.float32(one - b1p))
        return {"b1p": b1p, "b2p": b2p, "sparse_lr": sparse_lr, "dense_alpha": dense_alpha,
                "omb1": np.float32(one - self.b1), "omb2": np.float32(one - self.b2)}


class DeviceTwoTower:
    """Parameters + Adam slots on one HIP device."""

    def __init__(self, num_users, num_items, num_man, num_cat, d, learning_rate=0.001, seed=0, device=None,
                 init=None, device_init=False):
        """device_init=True draws the embedding tables' Keras
        uniform(-0.05, 0.05) init on the device (catalogue-sized tables, e.g.
        BASELINE c4's 50M x 128) instead of on the host."""
        _hrec.require_device()
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.d = int(d)
        self.sizes = {"user_emb": int(num_users), "item_emb": int(num_items), "man_emb": int(num_man),
                      "cat_emb": int(num_cat)}
        self.layout, self.n_dense = dense_layout(self.d)
        dev = self.device
        if init is None:
            init = keras_init(0 if device_init else num_users, 0 if device_init else num_items, num_man, num_cat, d,
                              seed)
            if device_init:
                g = torch.Generator(device=dev).manual_seed(int(seed))
                for name, rows in (("user_emb", num_users), ("item_emb", num_items)):
                    t = torch.empty((int(rows), self.d), dtype=torch.float32, device=dev)
                    init[name] = t.uniform_(-0.05, 0.05, generator=g)
        self.dense = torch.zeros(self.n_dense, dtype=torch.float32, device=dev)
        self.tensors = {}
        for name, (off, shape) in self.layout.items():
            view = self.dense[off: off + int(np.prod(shape))].view(*shape)
            view.copy_(torch.as_tensor(np.asarray(init[name], np.float32).reshape(shape)))
            self.tensors[name] = view
        for name in TABLES:
            t = init[name]
            self.tensors[name] = (t if isinstance(t, torch.Tensor) else
                                  torch.as_tensor(np.asarray(t, np.float32), device=dev)).contiguous()
        self.opt = AdamConfig(learning_rate)
        self.iterations = 0
        self.m_dense = torch.zeros_like(self.dense)
        self.v_dense = torch.zeros_like(self.dense)
        self.m_tab = {n: torch.zeros_like(self.tensors[n]) for n in TABLES}
        self.v_tab = {n: torch.zeros_like(self.tensors[n]) for n in TABLES}
        self.mark = {n: torch.full((self.tensors[n].shape[0],), -1, dtype=torch.int32, device=dev) for n in TABLES}
        self._ws = None
        # two-stream sparse Adam (hrec_adam_sparse_tables_phase) when every
        # table row is a whole number of 16-B vectors
        self._phased = (os.environ.get("HREC_TT_PHASED", "1") != "0"
                        and all(self.tensors[n].shape[1] % 4 == 0 for n in TABLES))
        if self._phased:
            self._side = torch.cuda.Stream(device=dev)
            self._ev_mark, self._ev_sweep = torch.cuda.Event(), torch.cuda.Event()
        self._refresh_params()

    def _refresh_params(self):
        self.params = _hrec.tt_params(self.d, self.tensors)

    # ---------------------------------------------------------- forward
    def item_vectors(self, item, man, cat, numeric, out=None):
        """Item tower over candidate rows; `out` ([n, d] f32) is written in
        place when given (catalogue precompute without a fresh allocation)."""
        return _hrec.tt_item_forward(self.params, item, man, cat, numeric, out=out)

    def user_vectors(self, user):
        return _hrec.tt_user_forward(self.params, user)

    def predict_rows(self, user, item, man, cat, numeric):
        """model.predict on per-row inputs: score[r] for row r."""
        return _hrec.tt_pair_score(self.user_vectors(user), self.item_vectors(item, man, cat, numeric))

    # ------------------------------------------------------------ train
    def train_step(self, user, item, man, cat, numeric, y):
        """One Keras train_step: forward + MSE + backward + Adam. Returns the
        device (sum_sq_err, sum_abs_err) pair of this batch."""
        B = user.numel()
        need = int(_hrec.lib().hrec_tt_train_workspace_bytes(self.d, B))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        c = self.opt.coefficients(self.iterations)
        adam = (c["sparse_lr"], self.opt.b1, c["omb1"], self.opt.b2, c["omb2"], self.opt.eps)
        idxs = (("user_emb", user), ("item_emb", item), ("man_emb", man), ("cat_emb", cat))
        if self._phased:
            # Two streams: the whole-table sweep of the rows this batch does
            # not touch (nearly all of the step's HBM bytes) runs on the side
            # stream while the forward / backward (which reads only touched
            # rows) runs here; the touched rows are stepped once their
            # gradients exist. Same bits as the one-stream grouped call.
            main = torch.cuda.current_stream(self.device)
            arg = _hrec.sparse_tables_arg([(self.tensors[n], self.m_tab[n], self.v_tab[n], idx, None, self.mark[n])
                                           for n, idx in idxs])
            _hrec.adam_sparse_tables_phase(arg, _hrec.SPARSE_MARK)
            self._ev_mark.record(main)
            with torch.cuda.stream(self._side):
                self._side.wait_event(self._ev_mark)
                _hrec.adam_sparse_tables_phase(arg, _hrec.SPARSE_SWEEP_UNTOUCHED, *adam)
                self._ev_sweep.record(self._side)
        gd, gu, gi, gm, gc = _hrec.tt_forward_backward(self.params, user, item, man, cat, numeric, y, self._ws)
        _hrec.adam_dense(self.dense, self.m_dense, self.v_dense, gd[: self.n_dense], c["dense_alpha"],
                         self.opt.b1, self.opt.b2, self.opt.eps)
        grads = (gu, gi, gm, gc)
        if self._phased:
            arg2 = _hrec.sparse_tables_arg([(self.tensors[n], self.m_tab[n], self.v_tab[n], idx, g, self.mark[n])
                                            for (n, idx), g in zip(idxs, grads)])
            _hrec.adam_sparse_tables_phase(arg2, _hrec.SPARSE_TOUCHED, *adam)
            main.wait_event(self._ev_sweep)
            _hrec.adam_sparse_tables_phase(arg, _hrec.SPARSE_UNMARK)
        else:
            # the four embedding tables' IndexedSlices updates in one grouped call
            tabs = [(self.tensors[n], self.m_tab[n], self.v_tab[n], idx, g, self.mark[n], torch.empty_like(g))
                    for (n, idx), g in zip(idxs, grads)]
            _hrec.adam_sparse_tables(tabs, *adam)
        self.iterations += 1
        return gd[self.n_dense:]

    # ------------------------------------------------------------ state
    def state_dict(self):
        out = {n: t.detach().cpu().numpy().copy() for n, t in self.tensors.items()}
        out["__iterations__"] = np.array(self.iterations)
        return out

    def optimizer_state(self):
        """Adam slots (Keras save_model's include_optimizer=True part)."""
        out = {"__opt_m_dense__": self.m_dense.cpu().numpy(), "__opt_v_dense__": self.v_dense.cpu().numpy()}
        for n in TABLES:
            out[f"__opt_m_{n}__"] = self.m_tab[n].cpu().numpy()
            out[f"__opt_v_{n}__"] = self.v_tab[n].cpu().numpy()
        return out

    def load_optimizer_state(self, state):
        """Restore what optimizer_state() saved (absent keys: slots stay zero)."""
        if "__opt_m_dense__" not in state:
            return False
        self.m_dense.copy_(torch.as_tensor(state["__opt_m_dense__"]))
        self.v_dense.copy_(torch.as_tensor(state["__opt_v_dense__"]))
        for n in TABLES:
            self.m_tab[n].copy_(torch.as_tensor(state[f"__opt_m_{n}__"]))
            self.v_tab[n].copy_(torch.as_tensor(state[f"__opt_v_{n}__"]))
        return True

    def snapshot(self):
        return {n: t.detach().clone() for n, t in self.tensors.items()}

    def restore(self, snap):
        for n, t in snap.items():
            self.tensors[n].copy_(t)
