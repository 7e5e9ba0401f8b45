"""Device plans for NeuralNetwork (fused MFMA MLP) and SupportVectorMachineModel.

MLP lowering (:class:`MlpPlan`): every layer becomes an A-operand fragment stream for
``v_mfma_f32_32x32x16_bf16`` (``precision="bf16"``, throughput path) or
``v_mfma_f32_32x32x2_f32`` (``precision="fp32"``, exact-fp32 parity path). Fragments are laid out
per (output tile t, k-step s, lane) so each lane issues one 16-byte (bf16) / 4-byte (fp32) load per
MFMA, and — for layers after the first — in the *permuted* k order in which the previous layer's
accumulator registers are consumed as the B operand (see ``csrc/mlp.hip``).
"""

from __future__ import annotations

import contextlib
from typing import List, Optional, Tuple

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..models.neural import NeuralEvaluator
from ..pmml import ir
from .plans import (EPI_AFFINE, LINKS, DevicePlan, NotLowerable, _addr, _epilogue, _label_table, apply_target_torch,
                    target_post)

ACT_CODES = {"identity": 0, "logistic": 1, "tanh": 2, "rectifier": 3, "exponential": 4, "reciprocal": 5,
             "square": 6, "Gauss": 7, "sine": 8, "cosine": 9, "Elliott": 10, "arctan": 11, "threshold": 12}
MT = 8  # max 32-unit tiles per layer (mirrors csrc/mlp.hip)
MAXL = 8  # max layers of the fused kernel
KMAX = 256  # max inputs per layer


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


def mlp_panels(meta, precision: str) -> np.ndarray:
    """The fused kernel's weight-panel schedule: one ``(offset, size)`` pair (16-byte units) per
    (layer, 32-unit output tile), in consumption order — every panel holds all k-step fragments
    of one output tile (``csrc/mlp.hip``)."""
    bf16 = precision == "bf16"
    esize, per_step = (2, 8) if bf16 else (4, 1)  # bytes per element, elements per lane per k-step
    out = []
    for kp, mp, _, w_off, _ in meta:
        ksteps = kp // (16 if bf16 else 2)
        tile_elems = ksteps * 64 * per_step
        for t in range(mp // 32):
            off = (w_off + t * tile_elems) * esize
            size = tile_elems * esize
            assert off % 16 == 0 and size % 16 == 0
            out.append((off // 16, size // 16))
    return np.array(out, dtype=np.int32)


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
        # K padded to whole k-step groups of 16 (csrc/mlp.hip runs one unrolled chain per group count)
        kp = ((K + 15) // 16) * 16 if L == 0 else prev_mp
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


def reg_kernel_ok(meta) -> bool:
    """Shapes the bf16 register-weight kernel runs (``csrc/mlp.hip::mlp_reg_kernel``): one or two
    hidden layers of at most 256 units over at most 256 inputs (their A fragments live in VGPRs)
    and an output layer of one 32-unit tile. ``meta`` rows: ``(kp, mp, mreal, w_off, b_off)``."""
    if len(meta) not in (2, 3):
        return False
    if any(kp > KMAX or mp > 32 * MT for kp, mp, *_ in meta):
        return False
    return meta[-1][1] == 32


class MlpPlan(DevicePlan):
    kind = "mlp"
    supports_direct = True
    _STATE = DevicePlan._STATE + ("weights", "biases", "layer_meta", "in_scale", "in_shift", "in_missing", "in_index",
                                  "n_in", "k0", "n_layers", "bf16", "out_a", "out_b", "final_norm", "n_out", "table",
                                  "is_classification", "panels", "n_panels", "contiguous", "target_stage", "reg_kernel")

    def __init__(self, compiled, device, precision: str = "fp32"):
        import torch

        super().__init__(compiled, device)
        ev: NeuralEvaluator = compiled.evaluator
        if precision not in ("bf16", "fp32"):
            raise ValueError("precision must be bf16 or fp32")
        self.bf16 = 1 if precision == "bf16" else 0
        layers, index = self._io(compiled, ev)
        if len(layers) > MAXL:
            raise NotLowerable(f"{len(layers)} layers > {MAXL} (fused kernel)")
        for W, b, act, thr, norm in layers:
            if W.shape[1] > 32 * MT:
                raise NotLowerable(f"layers wider than {32 * MT} units (fused kernel)")
        if self.n_in > KMAX:
            raise NotLowerable(f"more than {KMAX} inputs (fused kernel)")
        if self.n_out > 32:
            raise NotLowerable("more than 32 output neurons (fused kernel)")
        w, bias, meta = pack_mlp_weights([(W, b) for W, b, *_ in layers], precision)
        pan = mlp_panels(meta, precision)
        self.panels = self._t(pan.reshape(-1))
        self.n_panels = int(len(pan))
        identity = index == list(range(len(index)))
        self.contiguous = 1 if identity and self.n_in == meta[0][0] else 0
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
        self.reg_kernel = 1 if self.bf16 and reg_kernel_ok(meta) else 0

    def set_kernel(self, name: str) -> None:
        """Force the bf16 kernel: ``"reg"`` (register-weight, when the shape allows) or ``"panel"``."""
        if name not in ("reg", "panel"):
            raise ValueError(name)
        self.reg_kernel = 1 if name == "reg" and self.bf16 and reg_kernel_ok(self._meta()) else 0

    def _meta(self):
        lm = self.layer_meta.cpu().numpy()
        return [tuple(int(x) for x in row[:5]) for row in lm]

    def _io(self, compiled, ev):
        """Inputs (NormContinuous affine maps, missing replacements, active-field index), the
        dense layers, output normalisation and the target decode. Returns ``(layers, index)``."""
        if self.prep is not None:  # the input stages read raw columns: compile_plan adds the prepare pass
            raise NotLowerable("network plans read prepared inputs (MiningField / DataField treatment present)")
        nn = ev.nn
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
        for i, (W, b, act, thr, norm) in enumerate(layers):
            if act not in ACT_CODES:
                raise NotLowerable(f"activation {act!r}")
            if norm not in (None, "none") and i != len(layers) - 1:
                raise NotLowerable("hidden-layer normalisation is host-only")
        self.in_scale = self._t(np.array(scales, np.float32))
        self.in_shift = self._t(np.array(shifts, np.float32))
        self.in_missing = self._t(np.array(misses, np.float32))
        self.in_index = self._t(np.array(index, np.int32))
        last_norm = layers[-1][4]
        self.final_norm = {None: 0, "none": 0, "softmax": 1, "simplemax": 2}.get(last_norm)
        if self.final_norm is None:
            raise NotLowerable(f"output normalisation {last_norm!r}")
        self.n_out = layers[-1][0].shape[1]
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
            self.target_stage = None
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
            self.target_stage = target_post(tgt)
            if tgt is not None and self.target_stage is None:  # pure rescale: folded into the affine map
                a, b = a * tgt.rescale_factor, b * tgt.rescale_factor + tgt.rescale_constant
            self.out_a, self.out_b = a, b
            self.table = None
        return layers, index

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
        a.panels, a.n_panels, a.contiguous = ptr(self.panels), self.n_panels, self.contiguous
        a.prof = ptr(getattr(self, "prof", None))  # optional phase timers (scripts/kbench.py --mlp-prof)
        a.reg_kernel = self.reg_kernel
        a.epi = _epilogue(mode=EPI_AFFINE, a=self.out_a, b=self.out_b, table=self.table, tgt=self.target_stage)
        a.epi.score2, a.epi.valid2 = _addr(score2), _addr(valid2)
        a.score, a.valid, a.probs = _addr(score), _addr(valid), ptr(probs)
        check(self.lib.pmml_mlp_launch(stream_handle(stream), ctypes.byref(a), self.bf16), "mlp kernel")


_TORCH_ACT = {
    0: lambda z, t: z, 1: lambda z, t: z.sigmoid(), 2: lambda z, t: z.tanh(), 3: lambda z, t: z.clamp_min(0.0),
    4: lambda z, t: z.exp(), 5: lambda z, t: z.reciprocal(), 6: lambda z, t: z * z,
    7: lambda z, t: (-z * z).exp(), 8: lambda z, t: z.sin(), 9: lambda z, t: z.cos(),
    10: lambda z, t: z / (1.0 + z.abs()), 11: lambda z, t: z.atan() * 0.63661977236758134,
    12: lambda z, t: (z > t).to(z.dtype),
}


class GemmMlpPlan(MlpPlan):
    """NeuralNetworks beyond the fused kernel's register budget (more than 8 layers, 256 units per
    layer, 256 inputs or 32 outputs): every layer is one library GEMM on the matrix cores
    (``torch.addmm`` → hipBLASLt, fp32 or bf16 operands with fp32 accumulation) and the activations
    round-trip through HBM; input normalisation, activations, output normalisation and the target
    decode run as torch element-wise ops on the same stream. Slower than the fused kernel but no
    width / depth limit and no host fallback."""

    graph_small_batches = True  # several launches per call: HIP-graph replay for small batches (runtime/graphs.py)

    kind = "mlp_gemm"
    supports_direct = False
    _STATE = DevicePlan._STATE + ("in_scale", "in_shift", "in_missing", "in_index", "n_in", "bf16", "out_a", "out_b",
                                  "final_norm", "n_out", "table", "is_classification", "gemm_w", "gemm_b",
                                  "acts", "n_layers", "target_stage")

    def __init__(self, compiled, device, precision: str = "fp32"):
        import torch

        DevicePlan.__init__(self, compiled, device)
        ev: NeuralEvaluator = compiled.evaluator
        if precision not in ("bf16", "fp32"):
            raise ValueError("precision must be bf16 or fp32")
        self.bf16 = 1 if precision == "bf16" else 0
        layers, _ = self._io(compiled, ev)
        dt = torch.bfloat16 if self.bf16 else torch.float32
        self.n_layers = len(layers)
        # one flat buffer per kind (replicable as plan state): W_l stored [in, out] back to back
        self.gemm_w = torch.cat([torch.from_numpy(np.ascontiguousarray(W, np.float32)).reshape(-1)
                                 for W, *_ in layers]).to(dt).to(self.device)
        self.gemm_b = self._t(np.concatenate([np.asarray(b, np.float32) for _, b, *_ in layers]))
        self.acts = [(int(W.shape[0]), int(W.shape[1]), ACT_CODES[act], float(thr)) for W, b, act, thr, _ in layers]

    def launch(self, X, score, valid, stream=None, probs=None, score2=None, valid2=None) -> None:
        import torch

        ctx = torch.cuda.stream(stream) if stream is not None else torch.cuda.stream(torch.cuda.current_stream())
        with ctx:
            x = X.index_select(1, self.in_index.long())
            miss = torch.isnan(x)
            v = torch.where(miss, self.in_missing.expand_as(x), x * self.in_scale + self.in_shift)
            ok = ~torch.isnan(v).any(dim=1)
            h = torch.nan_to_num(v, nan=0.0)
            wo = bo = 0
            for k, m, act, thr in self.acts:
                W = self.gemm_w[wo: wo + k * m].view(k, m)
                b = self.gemm_b[bo: bo + m]
                wo += k * m
                bo += m
                z = torch.addmm(b.to(W.dtype), h.to(W.dtype), W).float()
                h = _TORCH_ACT[act](z, thr)
            if self.is_classification:
                if self.final_norm == 1:
                    p = torch.softmax(h, dim=1)
                elif self.final_norm == 2:
                    p = h / h.sum(dim=1, keepdim=True)
                else:
                    p = h
                lab = torch.argmax(torch.nan_to_num(p, nan=-float("inf")), dim=1)
                s = self.table[lab]
                ok = ok & ~torch.isnan(p).any(dim=1) & ~torch.isnan(s)
                if probs is not None:
                    probs.copy_(p)
            else:
                s = self.out_a * h[:, 0] + self.out_b
                ok = ok & torch.isfinite(s)
                s, ok = apply_target_torch(s, ok, self.target_stage)
            s = torch.where(ok, s, torch.full_like(s, float("nan")))
            for so, vo in ((score, valid), (score2, valid2)):
                if so is not None and not isinstance(so, int):
                    so.copy_(s)
                    vo.copy_(ok.to(torch.uint8))


def _ceil(x: int, m: int) -> int:
    return -(-x // m) * m


def fused_head_perm(K: int) -> np.ndarray:
    """Source unit of every storage position of the fused output layer's weight rows (K a multiple
    of 32): position g + 16 s + 8 h + e <- unit g + 16 s + 8 (e >> 2) + 4 h + (e & 3)."""
    q = np.arange(K)
    g, t = q - q % 32, q % 32
    s, h, e = t // 16, (t % 16) // 8, t % 8
    return (g + 16 * s + 8 * (e >> 2) + 4 * h + (e & 3)).astype(np.int64)


class WideMlpPlan(MlpPlan):
    """NeuralNetworks beyond the fused kernel (layers wider than 256 units, more than 8 layers or
    256 inputs) on ``gemm.hip``: an input-stage kernel (gather, NormContinuous, missing values,
    bf16), then ONE fused MFMA GEMM launch per layer — bias and activation in the epilogue,
    bf16 activations ping-pong through HBM — and an output-layer GEMM whose epilogue does the
    whole decode (output activation, softmax / simplemax, label table or affine + Target) into
    the score / valid / probability sinks. bf16 operands (precision bf16 / fp8) or exact fp32
    operands on ``v_mfma_f32_32x32x2f32`` (the default fp32 policy); fp32 accumulation."""

    graph_small_batches = False  # measured slower replayed (profiles/r3ag): few, large kernels; the graph's copies cost more

    kind = "mlp_wide"
    supports_direct = True
    _STATE = DevicePlan._STATE + ("in_scale", "in_shift", "in_missing", "in_index", "n_in", "out_a", "out_b",
                                  "final_norm", "n_out", "table", "is_classification", "target_stage", "wts", "bss",
                                  "dims", "k0", "bf16", "in_contig")
    ROWS = 256  # GEMM block rows (mirrors csrc/gemm.hip BM)

    def __init__(self, compiled, device, precision: str = "bf16"):
        import torch

        DevicePlan.__init__(self, compiled, device)
        ev: NeuralEvaluator = compiled.evaluator
        if precision not in ("bf16", "fp32"):
            raise ValueError("precision must be bf16 or fp32")
        self.bf16 = 1 if precision == "bf16" else 0
        layers, _ = self._io(compiled, ev)
        idx = self.in_index.cpu().numpy()
        # the input stage reads a contiguous, 16-byte aligned input map as two 16-byte loads per 8 inputs
        self.in_contig = int(len(idx) > 0 and idx[0] % 4 == 0 and bool((np.diff(idx) == 1).all()))
        if self.n_out > 1024:
            raise NotLowerable("more than 1024 output neurons")
        self.k0 = _ceil(max(self.n_in, 1), 64)
        if self.k0 > 16384:
            raise NotLowerable("more than 16384 network inputs (wide-layer input stage)")
        wts, bss, dims = [], [], []
        wo = bo = 0
        kp = self.k0
        for li, (W, b, act, thr, _) in enumerate(layers):
            k, m = W.shape
            head = li == len(layers) - 1
            mp = _ceil(m, 32) if head else _ceil(m, 256)  # output layer: 32-unit groups
            Wt = np.zeros((mp, kp), dtype=np.float32)
            Wt[:m, :k] = np.asarray(W, np.float32).T
            bias = np.zeros(mp, dtype=np.float32)
            bias[:m] = b
            wts.append(Wt.reshape(-1))
            bss.append(bias)
            dims.append((kp, mp, ACT_CODES[act], float(thr), wo, bo))
            wo += Wt.size
            bo += mp
            kp = mp
        self.wts = torch.from_numpy(np.concatenate(wts)).to(self._dtype()).to(self.device)
        self.bss = self._t(np.concatenate(bss))
        self.dims = dims

    gemm_flags = 0  # experiment bits ORed into GemmArgs.f32 (scripts/gemm_ab.py); the kernel rejects unknown bits
    # bf16: the last hidden layer and the output layer in one GEMM launch (gemm8_kernel<true>) — the
    # last hidden activations never reach HBM (profiles/r4f)
    fuse_head = True

    def _fused_head(self) -> bool:
        return (bool(self.fuse_head) and self.bf16 == 1 and len(self.dims) >= 2 and self.dims[-2][0] % 64 == 0
                and self.n_out <= 32)

    # bf16, <= 64 network inputs: the input stage runs inside the first layer's GEMM (gemm_k64_kernel<true>)
    fuse_input = False  # measured slower (the gather in the GEMM prologue: 1.41 vs 0.06 + 0.57 ms, profiles/r4v, r4y)

    def _fused_input(self, fused_head: bool) -> bool:
        """The first layer is a hidden layer launched on its own (not the fused last hidden layer)."""
        n_hidden = len(self.dims) - 1
        return (bool(self.fuse_input) and self.bf16 == 1 and self.k0 == 64 and self.gemm_flags == 0 and
                n_hidden >= 1 and not (fused_head and n_hidden == 1))

    def _head_weights(self):
        """The output layer's weights [32, K] with k permuted inside every 32-unit group as the
        fused epilogue consumes them: storage position 16 s + 8 h + e of a group holds unit
        16 s + 8 (e >> 2) + 4 h + (e & 3) — the unit an MFMA accumulator register (8 s + e) of lane
        half h carries (csrc/gemm.hip head_partial)."""
        w = getattr(self, "_whp", None)
        if w is None:
            import torch

            kp, mp, _, _, wo, _ = self.dims[-1]
            w = self._whp = self.wts[wo: wo + mp * kp].view(mp, kp)[:, torch.from_numpy(
                fused_head_perm(kp)).to(self.device)].contiguous()
        return w

    def _dtype(self):
        import torch

        return torch.bfloat16 if self.bf16 else torch.float32

    def launch(self, X, score, valid, stream=None, probs=None, score2=None, valid2=None) -> None:
        import ctypes

        import torch

        from ..ops._lib import GemmArgs, NnPrepArgs, check, ptr, stream_handle

        n = X.shape[0]
        if n == 0:
            return
        rows_p = _ceil(n, self.ROWS)
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        h = stream_handle(st)
        with torch.cuda.stream(st):
            widest = max(mp for _, mp, *_ in self.dims[:-1]) if len(self.dims) > 1 else 0
            dt = self._dtype()
            H0 = torch.empty((rows_p, self.k0), dtype=dt, device=self.device)
            bufs = [torch.empty((rows_p, widest), dtype=dt, device=self.device) for _ in range(2)] \
                if widest else []
            ok = torch.empty(rows_p, dtype=torch.uint8, device=self.device)
        p = NnPrepArgs()
        p.X, p.n_rows, p.rows_p, p.ldx, p.n_in = X.data_ptr(), n, rows_p, X.stride(0), self.n_in
        p.in_index, p.in_scale, p.in_shift = ptr(self.in_index), ptr(self.in_scale), ptr(self.in_shift)
        p.in_missing, p.H, p.ldh, p.k0, p.row_ok = ptr(self.in_missing), H0.data_ptr(), self.k0, self.k0, ok.data_ptr()
        p.f32 = 1 - self.bf16
        p.contig = getattr(self, "in_contig", 0)
        fused = self._fused_head()
        first = self._fused_input(fused)
        if not first:
            check(self.lib.pmml_nn_prep_launch(h, ctypes.byref(p)), "nn input stage")
        wbase, bbase, es = self.wts.data_ptr(), self.bss.data_ptr(), 2 if self.bf16 else 4
        extra = []
        cur, lda = H0, self.k0
        pending = None
        for li, (kp, mp, act, thr, wo, bo) in enumerate(self.dims):
            head = li == len(self.dims) - 1
            a = GemmArgs()
            a.A, a.Wt, a.bias, a.f32 = cur.data_ptr(), wbase + es * wo, bbase + 4 * bo, (1 - self.bf16) | self.gemm_flags
            a.rows, a.rows_p, a.K, a.Mp = n, rows_p, kp, mp
            a.lda, a.ldw, a.act, a.thr = lda, kp, act, thr
            if li == 0 and first:  # input stage + first hidden layer: one launch, no [rows, 64] round trip
                out = bufs[0]
                a.C, a.ldc = out.data_ptr(), out.stride(0)
                check(self.lib.pmml_nn_first_layer_launch(h, ctypes.byref(a), ctypes.byref(p)),
                      "nn input stage + first layer gemm")
                cur, lda = out, out.stride(0)
                continue
            if head:
                a.n_out, a.final_norm, a.row_ok = self.n_out, self.final_norm, ok.data_ptr()
                a.epi = _epilogue(mode=EPI_AFFINE, a=self.out_a, b=self.out_b, table=self.table, tgt=self.target_stage)
                a.epi.score2, a.epi.valid2 = _addr(score2), _addr(valid2)
                a.score, a.valid, a.probs = _addr(score), _addr(valid), ptr(probs)
                if pending is not None:  # last hidden layer + this one: one fused GEMM + the decode
                    whp = self._head_weights()
                    with torch.cuda.stream(st):
                        part = torch.empty((pending.Mp // 256) * rows_p * self.n_out, dtype=torch.float32,
                                           device=self.device)
                    extra.append(part)
                    check(self.lib.pmml_gemm_fused_head_launch(h, ctypes.byref(pending), ctypes.byref(a),
                                                               whp.data_ptr(), part.data_ptr()),
                          "nn fused last-hidden + output-layer gemm")
                elif mp <= 32:
                    check(self.lib.pmml_gemm_launch(h, ctypes.byref(a), 1), "nn output-layer gemm")
                else:  # > 32 outputs: one 32-unit group per launch into Z, then the wide decode
                    with torch.cuda.stream(st):
                        Z = torch.empty((rows_p, mp), dtype=torch.float32, device=self.device)
                    extra.append(Z)
                    for g in range(mp // 32):
                        ag = GemmArgs.from_buffer_copy(a)
                        ag.Wt, ag.bias = wbase + es * (wo + g * 32 * kp), bbase + 4 * (bo + 32 * g)
                        ag.Mp, ag.n_out = 32, min(32, self.n_out - 32 * g)
                        ag.C, ag.ldc = Z.data_ptr() + 4 * 32 * g, mp
                        check(self.lib.pmml_gemm_launch(h, ctypes.byref(ag), 1), "nn output-layer gemm (group)")
                    check(self.lib.pmml_nn_decode_wide(h, ctypes.byref(a), Z.data_ptr(), mp), "nn wide decode")
            elif fused and li == len(self.dims) - 2:
                pending = a  # its activations go straight into the output layer's MFMAs
            else:
                out = bufs[li & 1]
                a.C, a.ldc = out.data_ptr(), out.stride(0)
                check(self.lib.pmml_gemm_launch(h, ctypes.byref(a), 0), "nn layer gemm")
                cur, lda = out, out.stride(0)
        for t in [H0, ok] + bufs + extra:  # freed by the caching allocator only after this stream's work
            t.record_stream(st)


class SvmPlan(DevicePlan):
    """SupportVectorMachineModel on the fused kernel-evaluation + vote kernel (fp32)."""

    kind = "svm"
    supports_direct = True
    MMAX = 8
    _KERNELS = {"linear": 0, "polynomial": 1, "radialBasis": 2, "sigmoid": 3}
    _STATE = DevicePlan._STATE + ("target_stage", "in_index", "sv", "sv_norm", "coef", "intercept", "thr", "tgt", "alt", "n_in",
                                  "n_sv", "n_machines", "kernel_code", "classification", "gamma", "coef0", "degree",
                                  "max_wins", "n_classes", "table", "fmax", "n_svp")

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
        # >= 32 support vectors: the matrix-core kernel, support vectors padded to whole 32-vector
        # tiles (zero coefficients); fewer: the VALU kernel
        self.n_svp = -(-nsv // 32) * 32 if nsv >= 32 else 0
        Sp = np.zeros((max(1, nsv, self.n_svp), self.fmax), np.float32)
        Sp[:nsv, :F] = S
        Ap = np.zeros((max(1, nsv, self.n_svp), self.MMAX), np.float32)
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
        # PMML Target of a regression SVM (the oracle applies it to every regression model)
        self.target_stage = target_post(ev.target, force=True) if not self.classification else None
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
        a.epi = _epilogue(mode=EPI_AFFINE, table=self.table, tgt=self.target_stage)
        a.epi.score2, a.epi.valid2 = _addr(score2), _addr(valid2)
        a.score, a.valid, a.decision = _addr(score), _addr(valid), ptr(decision)
        check(self.lib.pmml_svm_launch(stream_handle(stream), ctypes.byref(a), self.fmax,
                                       getattr(self, "n_svp", 0)), "svm kernel")


def _pperm(i, h):
    """Row of a 32x32 MFMA accumulator held in register ``i`` by lane half ``h`` (csrc svm.hip)."""
    return (i & 3) + 8 * (i >> 2) + 4 * h


class SvmWidePlan(DevicePlan):
    """SupportVectorMachineModel beyond the fused kernel's limits — one-against-one over up to 256
    classes (up to 65535 machines: packed u16 vote counters), up to 128 vector fields, any number
    of support vectors — on ``svm_wide_kernel`` (``ops/csrc/svm.hip``): the decision function as two chained exact-fp32
    MFMA products (``G = S·xᵀ`` → kernel function on the accumulators → ``D = Aᵀ·K``) fused in
    one pass, votes in LDS; the [rows x support vectors] kernel matrix never leaves the registers.

    Host side: the support vectors, squared norms and dual coefficients are pre-swizzled so each
    lane streams contiguous 16-byte loads in the order the MFMA fragments consume them (the
    second product's B operand is the first product's accumulator register file, so the dual
    coefficients are permuted by the accumulator row map :func:`_pperm`). Parity: the oracle's
    ``models/svm.py::SvmEvaluator.decision_values/finish``."""

    kind = "svm_wide"
    supports_direct = True
    FMAXES = (16, 32, 64, 128)
    CMAX = 256  # packed u16 vote counters: TB x 128 dwords = 128 KiB of LDS
    _KERNELS = SvmPlan._KERNELS
    _STATE = DevicePlan._STATE + ("target_stage", "in_index", "svA", "coefA", "svnP", "intercept", "thr", "tgt", "alt", "n_in",
                                  "n_sv", "n_machines", "kernel_code", "classification", "gamma", "coef0", "degree",
                                  "max_wins", "n_classes", "table", "fmax", "mt", "n_tiles", "n_groups")

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
        self.fmax = next((b for b in self.FMAXES if F <= b), None)
        if self.fmax is None:
            raise NotLowerable(f"SVM with more than {self.FMAXES[-1]} vector fields (wide kernel)")
        M = len(sm.machines)
        if sm.representation == "Coefficients":
            S, A, kind = ev.linear_coef.T, np.eye(M), "linear"
        else:
            S, A, kind = ev.S, ev.A, sm.kernel.kind
        if kind not in self._KERNELS:
            raise NotLowerable(f"SVM kernel {kind!r}")
        self.classification = 1 if ev.kind == "classification" else 0
        # PMML Target of a regression SVM (the oracle applies it to every regression model)
        self.target_stage = target_post(ev.target, force=True) if not self.classification else None
        if not self.classification and M != 1:
            raise NotLowerable("regression SVM must have one machine")
        nsv = S.shape[0]
        self.n_sv, self.n_in, self.n_machines = nsv, F, M
        self.mt = 1 if M <= 32 else 2 if M <= 64 else 4
        self.n_groups = -(-M // (32 * self.mt))
        n_mtiles = self.n_groups * self.mt
        self.n_tiles = max(1, -(-nsv // 32))
        Sp = np.zeros((self.n_tiles * 32, self.fmax), np.float64)
        Sp[:nsv, :F] = S
        Ap = np.zeros((self.n_tiles * 32, n_mtiles * 32), np.float64)
        Ap[:nsv, :M] = A
        lane = np.arange(64)
        q = np.arange(self.fmax // 2)
        # svA[t, lane, q] = S[32t + (lane & 31), 2q + (lane >> 5)]
        rows = (np.arange(self.n_tiles)[:, None, None] * 32 + (lane & 31)[None, :, None])
        cols = 2 * q[None, None, :] + (lane >> 5)[None, :, None]
        self.svA = self._t(Sp[rows, cols].astype(np.float32))
        # coefA[t, mtile, lane, j] = A[32t + p(j, lane >> 5), 32 mtile + (lane & 31)]
        j = np.arange(16)
        sv_idx = (np.arange(self.n_tiles)[:, None, None, None] * 32
                  + _pperm(j[None, None, None, :], (lane >> 5)[None, None, :, None]))
        m_idx = np.arange(n_mtiles)[None, :, None, None] * 32 + (lane & 31)[None, None, :, None]
        self.coefA = self._t(Ap[sv_idx, m_idx].astype(np.float32))
        # svnP[t, h, i] = |S[32t + p(i, h)]|^2 (RBF)
        norms = (Sp.astype(np.float32).astype(np.float64) ** 2).sum(1).astype(np.float32)
        nidx = (np.arange(self.n_tiles)[:, None, None] * 32
                + _pperm(np.arange(16)[None, None, :], np.arange(2)[None, :, None]))
        self.svnP = self._t(norms[nidx])
        pad = n_mtiles * 32
        ic = np.zeros(pad, np.float32)
        ic[:M] = ev.b
        self.intercept = self._t(ic)
        self.in_index = self._t(np.array([compiled.active_fields.index(f) for f in fields], np.int32))
        self.kernel_code = self._KERNELS[kind]
        k = sm.kernel
        self.gamma, self.coef0, self.degree = float(k.gamma), float(k.coef0), float(k.degree)
        self.max_wins = 1 if sm.max_wins else 0
        thr = np.zeros(pad, np.float32)
        tgt = np.full(pad, -1, np.int32)
        alt = np.full(pad, -1, np.int32)
        if self.classification:
            cats = ev.categories
            if len(cats) > self.CMAX:
                raise NotLowerable(f"more than {self.CMAX} SVM classes (wide kernel vote counters)")
            if M > 0xFFFF:
                raise NotLowerable("more than 65535 SVM machines (u16 vote counters)")
            for m, mach in enumerate(sm.machines):
                thr[m] = mach.threshold if mach.threshold is not None else sm.threshold
                tgt[m] = cats.index(mach.target_category)
                if mach.alternate_target_category is not None:
                    alt[m] = cats.index(mach.alternate_target_category)
            self.table = self._t(_label_table(cats))
            self.n_classes = len(cats)
        else:
            self.table = None
            self.n_classes = 0
        self.thr, self.tgt, self.alt = self._t(thr), self._t(tgt), self._t(alt)

    def launch(self, X, score, valid, stream=None, probs=None, score2=None, valid2=None, decision=None) -> None:
        import ctypes

        from ..ops._lib import SvmWideArgs, check, ptr, stream_handle

        w = SvmWideArgs()
        a = w.s
        a.X = X.data_ptr()
        a.n_rows, a.n_feat, a.ldx, a.n_sv = X.shape[0], X.shape[1], X.stride(0), self.n_sv
        a.prep, a.in_index = ptr(self.prep), ptr(self.in_index)
        a.intercept, a.thr, a.tgt, a.alt = ptr(self.intercept), ptr(self.thr), ptr(self.tgt), ptr(self.alt)
        a.n_in, a.n_machines, a.kernel, a.classification = self.n_in, self.n_machines, self.kernel_code, \
            self.classification
        a.gamma, a.coef0, a.degree = self.gamma, self.coef0, self.degree
        a.max_wins, a.n_classes = self.max_wins, self.n_classes
        a.epi = _epilogue(mode=EPI_AFFINE, table=self.table, tgt=self.target_stage)
        a.epi.score2, a.epi.valid2 = _addr(score2), _addr(valid2)
        a.score, a.valid, a.decision = _addr(score), _addr(valid), ptr(decision)
        w.svA, w.coefA, w.svnP = ptr(self.svA), ptr(self.coefA), ptr(self.svnP)
        w.n_tiles, w.n_mtiles, w.n_groups = self.n_tiles, self.n_groups * self.mt, self.n_groups
        check(self.lib.pmml_svm_wide_launch(stream_handle(stream), ctypes.byref(w), self.fmax, self.mt),
              "svm wide kernel")


class SvmGemmPlan(DevicePlan):
    """SupportVectorMachineModel as two library GEMMs on the matrix cores (hipBLASLt, fp32):
    ``G = X·Sᵀ`` → kernel function (element-wise) → ``D = K·A + b`` (``A`` = dual coefficients of
    every machine over the shared support-vector set), then one-against-one / one-against-all
    votes as a tiny ``[machines, classes]`` product. Coalesced, MFMA-backed and without the fused
    kernel's limits (any number of machines, fields, support vectors); used when those limits bite.
    Reads prepared inputs (compile_plan puts a prepare-only derive pass in front when needed).
    Parity: the oracle's `models/svm.py::SvmEvaluator.decision_values/finish`."""

    graph_small_batches = True  # several launches per call: HIP-graph replay for small batches (runtime/graphs.py)

    kind = "svm_gemm"
    supports_direct = False
    ROW_CHUNK = 1 << 18  # bounds the [rows, n_sv] kernel matrix
    _STATE = DevicePlan._STATE + ("target_stage", "in_index", "S", "s_norm", "A", "b", "W_lin", "thr", "vote_t", "vote_a",
                                  "kernel_kind", "gamma", "coef0", "degree", "max_wins", "classification",
                                  "table", "coefficients")

    def __init__(self, compiled, device):
        import torch

        from ..models.svm import SvmEvaluator

        super().__init__(compiled, device)
        if self.prep is not None:
            raise NotLowerable("SvmGemmPlan reads prepared inputs (compile_plan adds the prepare pass)")
        ev: SvmEvaluator = compiled.evaluator
        sm = ev.sm
        fi = getattr(compiled, "field_index", None) or {f: i for i, f in enumerate(compiled.active_fields)}
        for f in ev.fields:
            if f not in fi:
                raise NotLowerable(f"SVM vector field {f!r} is not an input column")
        self.in_index = self._t(np.array([fi[f] for f in ev.fields], np.int64))
        self.coefficients = 1 if sm.representation == "Coefficients" else 0
        M = len(sm.machines)
        self.kernel_kind = "linear" if self.coefficients else sm.kernel.kind
        if self.kernel_kind not in ("linear", "polynomial", "radialBasis", "sigmoid"):
            raise NotLowerable(f"SVM kernel {self.kernel_kind!r}")
        k = sm.kernel
        self.gamma, self.coef0, self.degree = float(k.gamma), float(k.coef0), float(k.degree)
        self.W_lin = self._t(ev.linear_coef.astype(np.float32)) if self.coefficients else None
        self.S = self._t(ev.S.astype(np.float32)) if not self.coefficients else None
        self.s_norm = self._t((ev.S ** 2).sum(1).astype(np.float32)) if not self.coefficients else None
        self.A = self._t(ev.A.astype(np.float32)) if not self.coefficients else None
        self.b = self._t(ev.b.astype(np.float32))
        self.max_wins = 1 if sm.max_wins else 0
        self.classification = 1 if ev.kind == "classification" else 0
        # PMML Target of a regression SVM (the oracle applies it to every regression model)
        self.target_stage = target_post(ev.target, force=True) if not self.classification else None
        self.table = self.thr = self.vote_t = self.vote_a = None
        if self.classification:
            cats = ev.categories
            C = len(cats)
            thr = np.zeros(M, np.float32)
            vt = np.zeros((M, C), np.float32)
            va = np.zeros((M, C), np.float32)
            for m, mach in enumerate(sm.machines):
                thr[m] = mach.threshold if mach.threshold is not None else sm.threshold
                vt[m, cats.index(mach.target_category)] = 1.0
                if mach.alternate_target_category is not None:
                    va[m, cats.index(mach.alternate_target_category)] = 1.0
            self.thr, self.vote_t, self.vote_a = self._t(thr), self._t(vt), self._t(va)
            self.table = self._t(_label_table(cats))
        elif M != 1:
            raise NotLowerable("regression SVM must have one machine")
        del torch

    def _decision(self, x):
        import torch

        if self.coefficients:
            return torch.addmm(self.b, x, self.W_lin)
        G = x @ self.S.T
        kk = self.kernel_kind
        if kk == "radialBasis":
            d2 = (x * x).sum(1, keepdim=True) - 2.0 * G + self.s_norm[None, :]
            K = torch.exp(-self.gamma * d2.clamp_min(0.0))
        elif kk == "linear":
            K = G
        elif kk == "polynomial":
            K = torch.pow(self.gamma * G + self.coef0, self.degree)
        else:
            K = torch.tanh(self.gamma * G + self.coef0)
        return torch.addmm(self.b, K, self.A)

    def launch(self, X, score, valid, stream=None, probs=None, score2=None, valid2=None, **kw) -> None:
        import torch

        if self.device.type == "cuda":
            ctx = torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream(self.device))
        else:  # lowering dry run: the same tensor program on the host (CPU tests)
            ctx = contextlib.nullcontext()
        with ctx:
            n = X.shape[0]
            for lo in range(0, n, self.ROW_CHUNK):
                hi = min(n, lo + self.ROW_CHUNK)
                x = X[lo:hi].index_select(1, self.in_index)
                ok = ~torch.isnan(x).any(dim=1)
                D = self._decision(torch.nan_to_num(x, nan=0.0))
                if self.classification:
                    first = D < self.thr[None, :]
                    if self.max_wins:
                        first = ~first
                    votes = first.float() @ self.vote_t + (~first).float() @ self.vote_a
                    s = self.table[votes.argmax(dim=1)]  # ties -> first category, as np.argmax
                    ok = ok & ~torch.isnan(s)
                else:
                    s = D[:, 0]
                s = torch.where(ok, s, torch.full_like(s, float("nan")))
                if not self.classification:
                    s, ok = apply_target_torch(s, ok, self.target_stage)
                for so, vo in ((score, valid), (score2, valid2)):
                    if so is not None and not isinstance(so, int):
                        so[lo:hi].copy_(s)
                        vo[lo:hi].copy_(ok.to(torch.uint8))
