"""Build + load of the native HIP kernel library (``_pmml_kernels.so``) and its C ABI.

The kernels are plain HIP C++ compiled by ``hipcc --offload-arch=gfx950`` into one shared object
with ``extern "C"`` launchers that take a raw ``hipStream_t`` and a POD argument struct. Python
calls them through :mod:`ctypes` with ``torch`` tensor device pointers — no PyTorch C++ headers in
the build (incremental rebuilds take seconds), one HIP runtime in the process (the ``.so`` binds to the
``libamdhip64.so.7`` that ``torch`` already loaded, matched by SONAME).

On a machine with a GPU a missing / unloadable library is an error (:class:`KernelLibraryError`),
never a silent fallback.
"""

from __future__ import annotations

import ctypes
import glob
import logging
import os
import shutil
import subprocess
import threading
import time
from typing import List, Optional

logger = logging.getLogger(__name__)

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_PATH = os.path.join(HERE, "_pmml_kernels.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"


class KernelLibraryError(RuntimeError):
    pass


def sources() -> List[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _headers() -> List[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.h")))


def is_stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(p) > t for p in sources() + _headers())


def _deps(path: str, seen=None) -> List[str]:
    """``path`` plus every local header it includes (transitively, ``#include "x.h"``)."""
    import re

    seen = seen if seen is not None else set()
    if path in seen or not os.path.exists(path):
        return []
    seen.add(path)
    out = [path]
    with open(path) as fh:
        for m in re.finditer(r'^\s*#include\s+"([^"]+)"', fh.read(), re.M):
            out += _deps(os.path.join(os.path.dirname(path), m.group(1)), seen)
    return out


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise KernelLibraryError("hipcc not found (set HIPCC or install ROCm)")


def build(force: bool = False, verbose: bool = False, jobs: int = 0, incremental: bool = False) -> str:
    """Compile every ``csrc/*.hip`` for gfx950 and link ``_pmml_kernels.so`` (in-tree).
    ``incremental``: only recompile sources newer than their object (or than any header)."""
    if not force and not is_stale():
        return LIB_PATH
    jobs = jobs or max(1, min(8, os.cpu_count() or 1))
    cc = hipcc()
    objdir = os.path.join(HERE, "_build")
    os.makedirs(objdir, exist_ok=True)
    flags = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
             "-ffp-contract=fast", "-munsafe-fp-atomics"]
    procs = []
    objs = []
    # slowest translation units first (they bound the wall time of the parallel build)
    for src in sorted(sources(), key=lambda p: -os.path.getsize(p)):
        obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
        objs.append(obj)
        dep_t = max(os.path.getmtime(d) for d in _deps(src))
        if incremental and os.path.exists(obj) and os.path.getmtime(obj) > dep_t:
            continue
        cmd = [cc, *flags, "-c", src, "-o", obj]
        if verbose:
            logger.info("%s", " ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        while len([p for p in procs if p[1].poll() is None]) >= jobs:
            time.sleep(0.05)
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise KernelLibraryError(f"hipcc failed on {os.path.basename(src)}:\n{out.decode(errors='replace')}")
    tmp = LIB_PATH + ".tmp"
    cmd = [cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise KernelLibraryError(f"link failed:\n{r.stdout.decode(errors='replace')}")
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


# --------------------------------------------------------------------------- ctypes ABI

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_float = ctypes.c_float


class FieldPrep(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint32), ("lo", c_float), ("hi", c_float), ("missing_repl", c_float),
                ("invalid_repl", c_float), ("out_lo", c_float), ("out_hi", c_float), ("pad", c_float)]


class Epilogue(ctypes.Structure):
    _fields_ = [("mode", c_int), ("n_classes", c_int), ("a", c_float), ("b", c_float), ("thr", c_float),
                ("has_table", c_int), ("table", c_void_p), ("write_probs", c_int), ("link", c_int),
                ("score2", c_void_p), ("valid2", c_void_p), ("tgt", c_int), ("dflt", c_float),
                ("lo", ctypes.c_double), ("hi", ctypes.c_double), ("ta", ctypes.c_double), ("tb", ctypes.c_double)]


class TreeArgs(ctypes.Structure):
    _fields_ = [("X", c_void_p), ("n_rows", c_int), ("n_feat", c_int), ("ldx", c_int), ("pad0", c_int),
                ("prep", c_void_p), ("row_valid_in", c_void_p), ("blob", c_void_p), ("roots", c_void_p),
                ("leaves", c_void_p), ("tree_slot", c_void_p), ("n_trees", c_int), ("rec_words", c_int),
                ("chunk_trees", c_int), ("P", c_int), ("C", c_int), ("trees_per_split", c_int),
                ("general", c_int), ("variant", c_int), ("epi", Epilogue), ("score", c_void_p),
                ("valid", c_void_p), ("probs", c_void_p), ("partial", c_void_p), ("blob_nan", c_void_p),
                ("chunk_trees_nan", c_int), ("xcd_split", c_int), ("tree_w", c_void_p), ("acc_init", c_void_p),
                ("feat_map", c_void_p), ("rows_wide", c_int), ("mode", c_int), ("n_stage", c_int), ("pilp", c_int),
                ("prof", c_void_p), ("rank_thr", c_void_p), ("rank_cnt", c_void_p), ("rank_stride", c_int),
                ("leaf_onehot", c_int)]


class TextParseArgs(ctypes.Structure):
    _fields_ = [("buf", c_void_p), ("n_bytes", ctypes.c_longlong), ("starts", c_void_p), ("n_rows", c_int),
                ("n_cols", c_int), ("colmap", c_void_p), ("F", c_int), ("delim", ctypes.c_char), ("n_missing", c_int),
                ("missing", c_void_p), ("X", c_void_p), ("flagged", c_void_p), ("max_flagged", c_int),
                ("n_flagged", c_void_p)]


class MultiTreeArgs(ctypes.Structure):
    """tree.hip MultiTreeArgs: several pointer-layout ensembles (segments) over the same rows."""
    _fields_ = [("segs", c_void_p), ("X", c_void_p), ("S", c_void_p), ("V", c_void_p), ("P", c_void_p),
                ("poff", c_void_p), ("sidx", c_void_p), ("n_rows", c_int), ("n_feat", c_int), ("ldx", c_int),
                ("count", c_int)]


class SegArgs(ctypes.Structure):
    _fields_ = [("X", c_void_p), ("n_rows", c_int), ("ldx", c_int), ("S", c_void_p), ("V", c_void_p),
                ("P", c_void_p), ("coff", c_void_p), ("prog", c_void_p), ("pool", c_void_p), ("pc", c_void_p),
                ("weights", c_void_p), ("remap", c_void_p), ("table", c_void_p), ("K", c_int), ("C", c_int),
                ("method", c_int), ("classification", c_int), ("skip", c_int), ("tgt", c_int),
                ("lo", ctypes.c_double), ("hi", ctypes.c_double), ("ta", ctypes.c_double), ("tb", ctypes.c_double),
                ("dflt", ctypes.c_double), ("score", c_void_p), ("valid", c_void_p), ("score2", c_void_p),
                ("valid2", c_void_p), ("remap_stride", c_int), ("pad", c_int)]


class GroupedTreeArgs(ctypes.Structure):
    """tree_common.h GroupedTreeArgs: one wide-kernel launch over a mixed-model slice."""
    _fields_ = [("models", c_void_p), ("model_code", c_void_p), ("row_start", c_void_p), ("tile_start", c_void_p),
                ("Xg", c_void_p), ("perm", c_void_p), ("out_s", c_void_p), ("out_v", c_void_p), ("n_models", c_int),
                ("F", c_int)]


class LdsTreeArgs(ctypes.Structure):
    """tree_lds.hip LdsTreeArgs: the LDS-resident deep-forest walk."""
    _fields_ = [("t", TreeArgs), ("chunks", c_void_p), ("slice_chunk", c_void_p), ("n_slices", c_int),
                ("chunk_u4", c_int), ("rows", c_int), ("pad", c_int)]


class GenTreeArgs(ctypes.Structure):
    _fields_ = [("t", TreeArgs), ("nodes", c_void_p), ("children", c_void_p), ("preds", c_void_p),
                ("pool", c_void_p), ("trees", c_void_p), ("max_steps", c_int), ("pad", c_int),
                ("mix_mass", c_void_p), ("mix_w", c_void_p), ("mix_tab", c_void_p), ("remap", c_void_p),
                ("vcol", c_void_p)]


class HybridArgs(ctypes.Structure):
    _fields_ = [("t", TreeArgs), ("heads", c_void_p), ("head_words", c_int), ("tail_format", c_int)]


class ClusterArgs(ctypes.Structure):
    _fields_ = [("X", c_void_p), ("n_rows", c_int), ("n_feat", c_int), ("ldx", c_int), ("K", c_int),
                ("prep", c_void_p), ("centers", c_void_p), ("weights", c_void_p), ("scales", c_void_p),
                ("qweights", c_void_p), ("cfun", c_void_p), ("table", c_void_p), ("metric", c_int),
                ("similarity", c_int), ("p", c_float), ("pad", c_int), ("score", c_void_p), ("valid", c_void_p),
                ("label", c_void_p), ("affinity", c_void_p)]


class KnnArgs(ctypes.Structure):
    _fields_ = [("X", c_void_p), ("n_rows", c_int), ("n_feat", c_int), ("ldx", c_int), ("n_inst", c_int),
                ("prep", c_void_p), ("inst", c_void_p), ("weights", c_void_p), ("scales", c_void_p),
                ("qweights", c_void_p), ("cfun", c_void_p), ("inst_value", c_void_p), ("inst_class", c_void_p),
                ("class_table", c_void_p), ("metric", c_int), ("similarity", c_int), ("p", c_float), ("k", c_int),
                ("agg", c_int), ("threshold", c_float), ("epi", Epilogue), ("score", c_void_p),
                ("valid", c_void_p)]


class GemmArgs(ctypes.Structure):
    _fields_ = [("A", c_void_p), ("Wt", c_void_p), ("bias", c_void_p), ("C", c_void_p), ("rows", c_int),
                ("rows_p", c_int), ("K", c_int), ("Mp", c_int), ("lda", c_int), ("ldw", c_int), ("ldc", c_int),
                ("act", c_int), ("thr", c_float), ("n_out", c_int), ("final_norm", c_int), ("f32", c_int),
                ("row_ok", c_void_p), ("epi", Epilogue), ("score", c_void_p), ("valid", c_void_p),
                ("probs", c_void_p)]


class NnPrepArgs(ctypes.Structure):
    _fields_ = [("X", c_void_p), ("n_rows", c_int), ("rows_p", c_int), ("ldx", c_int), ("n_in", c_int),
                ("in_index", c_void_p), ("in_scale", c_void_p), ("in_shift", c_void_p), ("in_missing", c_void_p),
                ("H", c_void_p), ("ldh", c_int), ("k0", c_int), ("row_ok", c_void_p), ("f32", c_int),
                ("contig", c_int)]


class LinearArgs(ctypes.Structure):
    _fields_ = [("X", c_void_p), ("n_rows", c_int), ("n_feat", c_int), ("ldx", c_int), ("K", c_int),
                ("prep", c_void_p), ("W", c_void_p), ("bias", c_void_p), ("simplemax", c_int), ("pad", c_int),
                ("epi", Epilogue), ("score", c_void_p), ("valid", c_void_p), ("probs", c_void_p)]


class MlpArgs(ctypes.Structure):
    _fields_ = [("X", c_void_p), ("n_rows", c_int), ("n_feat", c_int), ("ldx", c_int), ("n_layers", c_int),
                ("in_scale", c_void_p), ("in_shift", c_void_p), ("in_missing", c_void_p), ("in_index", c_void_p),
                ("n_in", c_int), ("k0", c_int), ("weights", c_void_p), ("biases", c_void_p), ("layers", c_void_p),
                ("out_scale", c_float), ("out_shift", c_float), ("final_norm", c_int), ("n_out", c_int),
                ("epi", Epilogue), ("score", c_void_p), ("valid", c_void_p), ("probs", c_void_p),
                ("panels", c_void_p), ("n_panels", c_int), ("contiguous", c_int), ("prof", c_void_p),
                ("reg_kernel", c_int), ("pad_", c_int)]


class SvmArgs(ctypes.Structure):
    _fields_ = [("X", c_void_p), ("n_rows", c_int), ("n_feat", c_int), ("ldx", c_int), ("n_sv", c_int),
                ("prep", c_void_p), ("in_index", c_void_p), ("sv", c_void_p), ("sv_norm", c_void_p),
                ("coef", c_void_p), ("intercept", c_void_p), ("thr", c_void_p), ("tgt", c_void_p), ("alt", c_void_p),
                ("n_in", c_int), ("n_machines", c_int), ("kernel", c_int), ("classification", c_int),
                ("gamma", c_float), ("coef0", c_float), ("degree", c_float), ("max_wins", c_int),
                ("n_classes", c_int), ("pad", c_int), ("epi", Epilogue), ("score", c_void_p), ("valid", c_void_p),
                ("decision", c_void_p)]


class SvmWideArgs(ctypes.Structure):
    _fields_ = [("s", SvmArgs), ("svA", c_void_p), ("coefA", c_void_p), ("svnP", c_void_p), ("n_tiles", c_int),
                ("n_mtiles", c_int), ("n_groups", c_int), ("pad", c_int)]


class DeriveArgs(ctypes.Structure):
    _fields_ = [("X", c_void_p), ("n_rows", c_int), ("n_in", c_int), ("ldx", c_int), ("n_tile", c_int),
                ("prep", c_void_p), ("prog", c_void_p), ("pool", c_void_p), ("out_cols", c_void_p),
                ("n_insn", c_int), ("n_sel", c_int), ("out", c_void_p), ("row_ok", c_void_p)]


_ABI = {
    "pmml_segment_args_size": SegArgs,
    "pmml_textparse_args_size": TextParseArgs,
    "pmml_derive_args_size": DeriveArgs,
    "pmml_tree_args_size": TreeArgs,
    "pmml_tree_multi_args_size": MultiTreeArgs,
    "pmml_tree_general_args_size": GenTreeArgs,
    "pmml_tree_grouped_args_size": GroupedTreeArgs,
    "pmml_tree_lds_args_size": LdsTreeArgs,
    "pmml_tree_hybrid_args_size": HybridArgs,
    "pmml_cluster_args_size": ClusterArgs,
    "pmml_knn_args_size": KnnArgs,
    "pmml_gemm_args_size": GemmArgs,
    "pmml_nn_prep_args_size": NnPrepArgs,
    "pmml_linear_args_size": LinearArgs,
    "pmml_mlp_args_size": MlpArgs,
    "pmml_svm_args_size": SvmArgs,
    "pmml_svm_wide_args_size": SvmWideArgs,
}

_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


def load(auto_build: bool = True) -> ctypes.CDLL:
    """Load (building first if stale and ``hipcc`` is available) and ABI-check the library."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  -- bind to torch's HIP runtime before dlopen

        if auto_build and is_stale():
            try:
                build()
            except KernelLibraryError:
                # never run kernels older than their sources: a stale library silently computes
                # with an old ABI / old numerics. FJA_ALLOW_STALE_LIB=1 opts in explicitly.
                if not os.path.exists(LIB_PATH) or os.environ.get("FJA_ALLOW_STALE_LIB") != "1":
                    raise
                logger.warning("kernel sources newer than %s but rebuild failed; FJA_ALLOW_STALE_LIB=1: "
                               "using the existing library", LIB_PATH)
        if not os.path.exists(LIB_PATH):
            raise KernelLibraryError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        try:
            lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise KernelLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for fn, struct in _ABI.items():
            f = getattr(lib, fn, None)
            if f is None:
                continue
            f.restype = c_int
            got = f()
            if got != ctypes.sizeof(struct):
                raise KernelLibraryError(f"ABI mismatch: {fn}={got}, ctypes sizeof={ctypes.sizeof(struct)}")
        for name in ("pmml_tree_launch", "pmml_cluster_launch", "pmml_linear_launch", "pmml_mlp_launch",
                     "pmml_svm_launch"):
            f = getattr(lib, name, None)
            if f is not None:
                f.restype = c_int
        lib.pmml_tree_launch.argtypes = [c_void_p, ctypes.POINTER(TreeArgs), c_int, c_int, c_int, c_int]
        lib.pmml_host_device_ptr.argtypes = [c_void_p, ctypes.POINTER(c_void_p)]
        lib.pmml_host_device_ptr.restype = c_int
        lib.pmml_memcpy_async.argtypes = [c_void_p, c_void_p, ctypes.c_size_t, c_int, c_void_p]
        lib.pmml_memcpy_async.restype = c_int
        lib.pmml_cluster_launch.argtypes = [c_void_p, ctypes.POINTER(ClusterArgs)]
        lib.pmml_cluster_mfma_launch.restype = ctypes.c_int
        lib.pmml_cluster_mfma_launch.argtypes = [c_void_p, ctypes.POINTER(ClusterArgs), c_void_p, c_void_p,
                                                 ctypes.c_int, ctypes.c_int]
        lib.pmml_gemm_launch.restype = ctypes.c_int
        lib.pmml_gemm_launch.argtypes = [c_void_p, ctypes.POINTER(GemmArgs), ctypes.c_int]
        lib.pmml_nn_decode_wide.restype = ctypes.c_int
        lib.pmml_nn_decode_wide.argtypes = [c_void_p, ctypes.POINTER(GemmArgs), c_void_p, c_int]
        lib.pmml_nn_first_layer_launch.restype = ctypes.c_int
        lib.pmml_nn_first_layer_launch.argtypes = [c_void_p, ctypes.POINTER(GemmArgs), ctypes.POINTER(NnPrepArgs)]
        lib.pmml_gemm_fused_head_launch.restype = ctypes.c_int
        lib.pmml_gemm_fused_head_launch.argtypes = [c_void_p, ctypes.POINTER(GemmArgs), ctypes.POINTER(GemmArgs),
                                                    c_void_p, c_void_p]
        lib.pmml_nn_prep_launch.restype = ctypes.c_int
        lib.pmml_nn_prep_launch.argtypes = [c_void_p, ctypes.POINTER(NnPrepArgs)]
        lib.pmml_knn_launch.restype = ctypes.c_int
        lib.pmml_knn_launch.argtypes = [c_void_p, ctypes.POINTER(KnnArgs), c_void_p, c_void_p, ctypes.c_int,
                                        ctypes.c_int]
        lib.pmml_linear_launch.argtypes = [c_void_p, ctypes.POINTER(LinearArgs)]
        if hasattr(lib, "pmml_mlp_launch"):
            lib.pmml_mlp_launch.argtypes = [c_void_p, ctypes.POINTER(MlpArgs), c_int]
        if hasattr(lib, "pmml_svm_launch"):
            lib.pmml_svm_launch.argtypes = [c_void_p, ctypes.POINTER(SvmArgs), c_int, c_int]
        if hasattr(lib, "pmml_svm_wide_launch"):
            lib.pmml_svm_wide_launch.restype = c_int
            lib.pmml_svm_wide_launch.argtypes = [c_void_p, ctypes.POINTER(SvmWideArgs), c_int, c_int]
        lib.pmml_tree_general_launch.argtypes = [c_void_p, ctypes.POINTER(GenTreeArgs)]
        lib.pmml_tree_general_launch.restype = c_int
        lib.pmml_tree_hybrid_launch.argtypes = [c_void_p, ctypes.POINTER(HybridArgs), c_int, c_int]
        lib.pmml_tree_hybrid_launch.restype = c_int
        lib.pmml_derive_launch.argtypes = [c_void_p, ctypes.POINTER(DeriveArgs)]
        lib.pmml_derive_launch.restype = c_int
        lib.pmml_mask_invalid.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int]
        lib.pmml_mask_invalid.restype = c_int
        lib.pmml_host_register.argtypes = [c_void_p, ctypes.c_size_t, ctypes.c_uint]
        lib.pmml_host_register.restype = c_int
        lib.pmml_host_unregister.argtypes = [c_void_p]
        lib.pmml_host_unregister.restype = c_int
        lib.pmml_segment_reduce.argtypes = [c_void_p, ctypes.POINTER(SegArgs)]
        lib.pmml_tree_pointer_multi.argtypes = [c_void_p, ctypes.POINTER(MultiTreeArgs), c_int, c_int]
        lib.pmml_tree_pointer_multi.restype = c_int
        lib.pmml_segment_reduce.restype = c_int
        lib.pmml_tree_launch_many.argtypes = [c_void_p, c_void_p, c_void_p, c_int]
        lib.pmml_tree_launch_many.restype = c_int
        lib.pmml_text_rows_count.argtypes = [c_void_p, c_void_p, ctypes.c_longlong, c_void_p]
        lib.pmml_text_rows_count.restype = c_int
        lib.pmml_text_rows_write.argtypes = [c_void_p, c_void_p, ctypes.c_longlong, c_void_p, c_void_p]
        lib.pmml_text_rows_write.restype = c_int
        lib.pmml_text_parse.argtypes = [c_void_p, ctypes.POINTER(TextParseArgs)]
        lib.pmml_text_parse.restype = c_int
        lib.pmml_group_rows.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                                        c_void_p, c_void_p]
        lib.pmml_group_rows.restype = c_int
        lib.pmml_ungroup.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                     c_void_p]
        lib.pmml_ungroup.restype = c_int
        lib.pmml_group_slice.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                                         c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p]
        lib.pmml_group_slice.restype = c_int
        lib.pmml_tree_launch_grouped.argtypes = [c_void_p, c_void_p, c_int, ctypes.POINTER(GroupedTreeArgs), c_int,
                                                 c_int]
        lib.pmml_tree_launch_grouped.restype = c_int
        lib.pmml_tree_lds_launch.argtypes = [c_void_p, ctypes.POINTER(LdsTreeArgs)]
        lib.pmml_tree_lds_launch.restype = c_int
        lib.pmml_tree_lds_bytes.argtypes = [c_int, c_int, c_int, c_int, c_int]
        lib.pmml_tree_lds_bytes.restype = ctypes.c_longlong
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise KernelLibraryError(f"{what} failed with code {rc}")


def ptr(t) -> Optional[int]:
    """Device pointer of a tensor (None → NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(stream=None) -> int:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def host_device_ptr(t) -> Optional[int]:
    """Device-visible address of a pinned host tensor (zero-copy), or None if not mapped."""
    if t is None or not t.is_pinned():
        return None
    lib = load()
    dev = c_void_p()
    rc = lib.pmml_host_device_ptr(c_void_p(t.data_ptr()), ctypes.byref(dev))
    if rc != 0 or not dev.value:
        return None
    return int(dev.value)
