"""Device plans for NeuralNetwork (fused MFMA MLP) and SupportVectorMachineModel.

MLP lowering (:class:`MlpPlan`): every layer becomes an A-operand fragment stream for
``v_mfma_f32_32x32x16_bf16`` (``precision="bf16"``, throughput path) or
``v_mfma_f32_32x32x2_f32`` (``precision="fp32"``, exact-fp32 parity path). Fragments are laid out
per (output tile t, k-step s, lane) so each lane issues one 16-byte (bf16) / 4-byte (fp32) load per
MFMA, and — for layers after the first — in the *permuted* k order in which the previous layer's
accumulator registers are consumed as the B operand (see ``csrc/mlp.hip``).
"""

from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..models.neural import NeuralEvaluator
from ..pmml import ir
from .plans import EPI_AFFINE, LINKS, DevicePlan, NotLowerable, _addr, _epilogue, _label_table

ACT_CODES = {"identity": 0, "logistic": 1, "tanh": 2, "rectifier": 3, "exponential": 4, "reciprocal": 5,
             "square": 6, "Gauss": 7, "sine": 8, "cosine": 9, "Elliott": 10, "arctan": 11, "threshold": 12}
MT = 8  # max 32-unit tiles per layer (mirrors csrc/mlp.hip)
MAXL = 4


def _affine_of(ex) -> Tuple[float, float, float]:
    """(scale, shift, missing) of a 2-point NormContinuous / FieldRef input."""
    if isinstance(ex, ir.FieldRef):
        miss = float(ex.map_missing_to) if ex.map_missing_to is not None else float("nan")
        return 1.0, 0.0, miss
    if isinstance(ex, ir.NormContinuous):
        if len(ex.norms) != 2 or ex.outliers != "asIs":
            raise NotLowerable("only 2-point NormContinuous inputs (outliers=asIs) are lowered")
        (o0, n0), (o1, n1) = (ex.norms[0].orig, ex.norms[0].norm), (ex.norms[1].orig, ex.norms[1].norm)
        sc = (n1 - n0) / (o1 - o0)
        miss = float(ex.map_missing_to) if ex.map_missing_to is not None else float("nan")
        return sc, n0 - o0 * sc, miss
    raise NotLowerable(f"NeuralInput expression {type(ex).__name__} is host-only")


def pack_mlp_weights(layers: List[Tuple[np.ndarray, np.ndarray]], precision: str):
    """Pack ``[(W[in, out], b[out])]`` into MFMA A-fragments.

    Returns ``(weights (flat), biases (flat), meta rows [kp, mp, mreal, w_off, b_off])``."""
    frags: List[np.ndarray] = []
    biases: List[np.ndarray] = []
    meta = []
    w_off = 0
    b_off = 0
    bf16 = precision == "bf16"
    kstep = 16 if bf16 else 2
    prev_mp = None
    for L, (W, b) in enumerate(layers):
        K, M = W.shape
        mp = ((M + 31) // 32) * 32
        kp = ((K + kstep - 1) // kstep) * kstep if L == 0 else prev_mp
        if L == 0 and bf16:
            kp = ((K + 15) // 16) * 16
        At = np.zeros((mp, kp))  # Wᵀ padded: [units, inputs]
        At[:M, :K] = W.T
        ksteps = kp // kstep
        mtiles = mp // 32
        lane = np.arange(64)
        m_idx = lane & 31
        hh = lane >> 5
        if bf16:
            out = np.zeros((mtiles, ksteps, 64, 8))
            j = np.arange(8)
            for t in range(mtiles):
                for s in range(ksteps):
                    if L == 0:
                        kk = 16 * s + 8 * hh[:, None] + j[None, :]
                    else:
                        tp, sp = s // 2, s % 2
                        kk = 32 * tp + 16 * sp + 8 * (j[None, :] >> 2) + 4 * hh[:, None] + (j[None, :] & 3)
                    out[t, s] = At[32 * t + m_idx[:, None], kk]
        else:
            out = np.zeros((mtiles, ksteps, 64))
            for t in range(mtiles):
                for s in range(ksteps):
                    if L == 0:
                        kk = 2 * s + hh
                    else:
                        tp, r = s // 16, s % 16
                        kk = 32 * tp + (r & 3) + 8 * (r >> 2) + 4 * hh
                    out[t, s] = At[32 * t + m_idx, kk]
        frags.append(out.reshape(-1))
        bb = np.zeros(mp)
        bb[:M] = b
        biases.append(bb)
        meta.append((kp, mp, M, w_off, b_off))
        w_off += out.size
        b_off += mp
        prev_mp = mp
    return np.concatenate(frags), np.concatenate(biases), meta


class MlpPlan(DevicePlan):
    kind = "mlp"
    supports_direct = True
    _STATE = DevicePlan._STATE + ("weights", "biases", "layer_meta", "in_scale", "in_shift", "in_missing", "in_index",
                                  "n_in", "k0", "n_layers", "bf16", "out_a", "out_b", "final_norm", "n_out", "table",
                                  "is_classification")

    def __init__(self, compiled, device, precision: str = "bf16"):
        import torch

        super().__init__(compiled, device)
        ev: NeuralEvaluator = compiled.evaluator
        if precision not in ("bf16", "fp32"):
            raise ValueError("precision must be bf16 or fp32")
        self.bf16 = 1 if precision == "bf16" else 0
        nn = ev.nn
        # inputs
        scales, shifts, misses, index = [], [], [], []
        for inp in nn.inputs:
            ex = inp.derived.expression
            field = ex.field
            if field not in compiled.active_fields:
                raise NotLowerable(f"NeuralInput on non-active field {field!r}")
            sc, sh, miss = _affine_of(ex)
            scales.append(sc)
            shifts.append(sh)
            misses.append(miss)
            index.append(compiled.active_fields.index(field))
        self.n_in = len(index)
        layers = ev.dense_layers()
        if len(layers) > MAXL:
            raise NotLowerable(f"{len(layers)} layers > {MAXL}")
        for i, (W, b, act, thr, norm) in enumerate(layers):
            if act not in ACT_CODES:
                raise NotLowerable(f"activation {act!r}")
            if W.shape[1] > 32 * MT:
                raise NotLowerable("layers wider than 256 units are host-only")
            if norm not in (None, "none") and i != len(layers) - 1:
                raise NotLowerable("hidden-layer normalisation is host-only")
        if self.n_in > 256:
            raise NotLowerable("more than 256 inputs")
        w, bias, meta = pack_mlp_weights([(W, b) for W, b, *_ in layers], precision)
        self.n_layers = len(layers)
        lm = np.zeros((self.n_layers, 8), dtype=np.int32)
        for i, ((kp, mp, mreal, wo, bo), (_, _, act, thr, _)) in enumerate(zip(meta, layers)):
            lm[i, :6] = [kp, mp, mreal, wo, bo, ACT_CODES[act]]
            lm[i, 6] = np.float32(thr).view(np.int32)
        self.k0 = meta[0][0]
        wt = torch.from_numpy(w.astype(np.float32))
        self.weights = (wt.to(torch.bfloat16) if self.bf16 else wt).to(self.device)
        self.biases = self._t(bias.astype(np.float32))
        self.layer_meta = self._t(lm)
        self.in_scale = self._t(np.array(scales, np.float32))
        self.in_shift = self._t(np.array(shifts, np.float32))
        self.in_missing = self._t(np.array(misses, np.float32))
        self.in_index = self._t(np.array(index, np.int32))
        last_norm = layers[-1][4]
        self.final_norm = {None: 0, "none": 0, "softmax": 1, "simplemax": 2}.get(last_norm)
        if self.final_norm is None:
            raise NotLowerable(f"output normalisation {last_norm!r}")
        self.n_out = layers[-1][0].shape[1]
        if self.n_out > 32:
            raise NotLowerable("more than 32 output neurons")
        out_neurons = [n.id for n in nn.layers[-1].neurons]
        self.is_classification = ev.kind == "classification"
        if self.is_classification:
            labels = [None] * self.n_out
            for o in nn.outputs:
                ex = o.derived.expression
                if not isinstance(ex, ir.NormDiscrete) or o.neuron not in out_neurons:
                    raise NotLowerable("classification outputs must be NormDiscrete on output neurons")
                labels[out_neurons.index(o.neuron)] = ex.value
            self.table = self._t(_label_table([x if x is not None else "nan" for x in labels]))
            self.out_a, self.out_b = 1.0, 0.0
        else:
            if self.n_out != 1 or len(nn.outputs) != 1 or nn.outputs[0].neuron != out_neurons[0]:
                raise NotLowerable("regression NN must have one output neuron")
            ex = nn.outputs[0].derived.expression
            if isinstance(ex, ir.FieldRef):
                a, b = 1.0, 0.0
            elif isinstance(ex, ir.NormContinuous) and len(ex.norms) == 2:
                (o0, n0), (o1, n1) = (ex.norms[0].orig, ex.norms[0].norm), (ex.norms[1].orig, ex.norms[1].norm)
                a = (o1 - o0) / (n1 - n0)
                b = o0 - n0 * a
            else:
                raise NotLowerable("regression NeuralOutput must be FieldRef or 2-point NormContinuous")
            tgt = ev.target
            if tgt is not None:
                if tgt.min is not None or tgt.max is not None or tgt.cast_integer:
                    raise NotLowerable("Target min/max/castInteger is host-only")
                a, b = a * tgt.rescale_factor, b * tgt.rescale_factor + tgt.rescale_constant
            self.out_a, self.out_b = a, b
            self.table = None

    def launch(self, X, score, valid, stream=None, probs=None, score2=None, valid2=None) -> None:
        import ctypes

        from ..ops._lib import MlpArgs, check, ptr, stream_handle

        a = MlpArgs()
        a.X = X.data_ptr()
        a.n_rows, a.n_feat, a.ldx, a.n_layers = X.shape[0], X.shape[1], X.stride(0), self.n_layers
        a.in_scale, a.in_shift, a.in_missing = ptr(self.in_scale), ptr(self.in_shift), ptr(self.in_missing)
        a.in_index, a.n_in, a.k0 = ptr(self.in_index), self.n_in, self.k0
        a.weights, a.biases, a.layers = ptr(self.weights), ptr(self.biases), ptr(self.layer_meta)
        a.out_scale, a.out_shift, a.final_norm, a.n_out = self.out_a, self.out_b, self.final_norm, self.n_out
        a.epi = _epilogue(mode=EPI_AFFINE, a=self.out_a, b=self.out_b, table=self.table)
        a.epi.score2, a.epi.valid2 = _addr(score2), _addr(valid2)
        a.score, a.valid, a.probs = _addr(score), _addr(valid), ptr(probs)
        check(self.lib.pmml_mlp_launch(stream_handle(stream), ctypes.byref(a), self.bf16), "mlp kernel")


class SvmPlan(DevicePlan):
    """SupportVectorMachineModel on the fused kernel-evaluation + vote kernel (fp32)."""

    kind = "svm"
    supports_direct = True
    MMAX = 8
    _KERNELS = {"linear": 0, "polynomial": 1, "radialBasis": 2, "sigmoid": 3}
    _STATE = DevicePlan._STATE + ("in_index", "sv", "sv_norm", "coef", "intercept", "thr", "tgt", "alt", "n_in",
                                  "n_sv", "n_machines", "kernel_code", "classification", "gamma", "coef0", "degree",
                                  "max_wins", "n_classes", "table", "fmax")

    def __init__(self, compiled, device):
        from ..models.svm import SvmEvaluator

        super().__init__(compiled, device)
        ev: SvmEvaluator = compiled.evaluator
        sm = ev.sm
        fields = ev.fields
        for f in fields:
            if f not in compiled.active_fields:
                raise NotLowerable(f"SVM vector field {f!r} is not an active field")
        F = len(fields)
        self.fmax = next((b for b in (8, 16, 32, 64) if F <= b), None)
        if self.fmax is None:
            raise NotLowerable("SVM with more than 64 vector fields is host-only")
        M = len(sm.machines)
        if M > self.MMAX:
            raise NotLowerable(f"{M} SVM machines > {self.MMAX}")
        if sm.representation == "Coefficients":
            # linear kernel with primal coefficients: one "support vector" per machine
            S = ev.linear_coef.T  # [M, F]
            A = np.eye(M)
            kind = "linear"
        else:
            S = ev.S
            A = ev.A
            kind = sm.kernel.kind
        nsv = S.shape[0]
        Sp = np.zeros((max(1, nsv), self.fmax), np.float32)
        Sp[:nsv, :F] = S
        Ap = np.zeros((max(1, nsv), self.MMAX), np.float32)
        Ap[:nsv, :M] = A
        self.n_sv, self.n_in, self.n_machines = nsv, F, M
        self.sv = self._t(Sp)
        self.sv_norm = self._t((Sp.astype(np.float64) ** 2).sum(1).astype(np.float32))
        self.coef = self._t(Ap)
        ic = np.zeros(self.MMAX, np.float32)
        ic[:M] = ev.b
        self.intercept = self._t(ic)
        self.in_index = self._t(np.array([compiled.active_fields.index(f) for f in fields], np.int32))
        self.kernel_code = self._KERNELS[kind]
        k = sm.kernel
        self.gamma, self.coef0, self.degree = float(k.gamma), float(k.coef0), float(k.degree)
        self.max_wins = 1 if sm.max_wins else 0
        thr = np.zeros(self.MMAX, np.float32)
        tgt = np.zeros(self.MMAX, np.int32)
        alt = np.full(self.MMAX, -1, np.int32)
        self.classification = 1 if ev.kind == "classification" else 0
        if self.classification:
            cats = ev.categories
            if len(cats) > 16:
                raise NotLowerable("more than 16 SVM classes")
            for m, mach in enumerate(sm.machines):
                thr[m] = mach.threshold if mach.threshold is not None else sm.threshold
                tgt[m] = cats.index(mach.target_category)
                if mach.alternate_target_category is not None:
                    alt[m] = cats.index(mach.alternate_target_category)
            self.table = self._t(_label_table(cats))
            self.n_classes = len(cats)
        else:
            if M != 1:
                raise NotLowerable("regression SVM must have one machine")
            self.table = None
            self.n_classes = 0
        self.thr, self.tgt, self.alt = self._t(thr), self._t(tgt), self._t(alt)

    def launch(self, X, score, valid, stream=None, probs=None, score2=None, valid2=None, decision=None) -> None:
        import ctypes

        from ..ops._lib import SvmArgs, check, ptr, stream_handle

        a = SvmArgs()
        a.X = X.data_ptr()
        a.n_rows, a.n_feat, a.ldx, a.n_sv = X.shape[0], X.shape[1], X.stride(0), self.n_sv
        a.prep, a.in_index, a.sv, a.sv_norm = ptr(self.prep), ptr(self.in_index), ptr(self.sv), ptr(self.sv_norm)
        a.coef, a.intercept, a.thr, a.tgt, a.alt = (ptr(self.coef), ptr(self.intercept), ptr(self.thr),
                                                     ptr(self.tgt), ptr(self.alt))
        a.n_in, a.n_machines, a.kernel, a.classification = self.n_in, self.n_machines, self.kernel_code, \
            self.classification
        a.gamma, a.coef0, a.degree = self.gamma, self.coef0, self.degree
        a.max_wins, a.n_classes = self.max_wins, self.n_classes
        a.epi = _epilogue(mode=EPI_AFFINE, table=self.table)
        a.epi.score2, a.epi.valid2 = _addr(score2), _addr(valid2)
        a.score, a.valid, a.decision = _addr(score), _addr(valid), ptr(decision)
        check(self.lib.pmml_svm_launch(stream_handle(stream), ctypes.byref(a), self.fmax), "svm kernel")
