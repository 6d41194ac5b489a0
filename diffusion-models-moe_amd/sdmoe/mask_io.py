"""On-disk mask / expert-list formats of the reference, and the bit-packed device layout used here.

Reference formats (SURVEY §8b "On-disk inputs"):
  * timestep_{t}_layer_{l}.json  : JSON list of removed expert ids (RemoveExperts, remove_skilled_experts.py:13-19)
                                   or a list of [row, col] neuron-weight indices (WandaRemoveNeurons, :20-28)
  * timestep_{t}_layer_{l}.pkl   : pickled scipy.sparse.csr_matrix (modularity/wanda.py:169-173) or np.matrix /
                                   ndarray (benchmarks/save_union_experts.py:123-126) binary [C, 4C] Wanda mask
  * param_split/<ffn>.proj.weight: torch.save(list[int]) expert labels (moefication/moe_utils.py:54-61)
Pickles are read with a restricted unpickler that only resolves numpy / scipy.sparse reconstruction helpers, so
a mask file cannot execute arbitrary code. The native format is `.npz` with the mask bit-packed along the last
dim (np.packbits(..., bitorder='little')), which is exactly the device layout the GEMM's B-load consumes:
bit j of byte (n*K + k)/8 is W[n, k].
"""
from __future__ import annotations

import io
import json
import os
import pickle

import numpy as np

_ALLOWED = {
    ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy", "matrix"),
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy.matrixlib.defmatrix", "matrix"),
    ("scipy.sparse._csr", "csr_matrix"), ("scipy.sparse.csr", "csr_matrix"),
    ("scipy.sparse._csr", "csr_array"), ("scipy.sparse._coo", "coo_matrix"), ("scipy.sparse._csc", "csc_matrix"),
    ("builtins", "tuple"), ("builtins", "list"), ("builtins", "dict"), ("collections", "OrderedDict"),
    ("copyreg", "_reconstructor"), ("builtins", "object"),
}


class _MaskUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a mask file")


def load_mask_pickle(path) -> np.ndarray:
    """Dense 0/1 int64 mask from a reference .pkl (csr_matrix or dense matrix), restricted unpickling."""
    with open(path, "rb") as f:
        obj = _MaskUnpickler(io.BytesIO(f.read())).load()
    if hasattr(obj, "toarray"):
        obj = obj.toarray()
    return (np.asarray(obj) != 0).astype(np.int64)


def pack_mask(mask) -> np.ndarray:
    m = np.asarray(mask)
    if m.shape[-1] % 8:
        raise ValueError("mask inner dim must be a multiple of 8")
    return np.packbits((m != 0).astype(np.uint8), axis=-1, bitorder="little")


def unpack_mask(bits, cols) -> np.ndarray:
    return np.unpackbits(np.asarray(bits, dtype=np.uint8), axis=-1, count=cols, bitorder="little").astype(np.int64)


def load_labels(path) -> list:
    """Expert labels written by ParamSplit.save (moe_utils.py:54-61: torch.save([x for x in kmeans.labels_])), i.e.
    a list of numpy int32/int64 scalars, or of Python ints. torch.load(weights_only=True) with only numpy's
    scalar reconstructor and integer dtypes added to its allow-list: nothing else in the file can execute."""
    import torch
    core = getattr(np, "_core", None) or np.core
    allowed = [core.multiarray.scalar, np.dtype]
    for name in ("Int8DType", "Int16DType", "Int32DType", "Int64DType", "UInt8DType", "UInt16DType", "UInt32DType",
                 "UInt64DType", "LongDType", "ULongDType", "LongLongDType", "ULongLongDType"):
        t = getattr(np.dtypes, name, None)
        if t is not None:
            allowed.append(t)
    with torch.serialization.safe_globals(allowed):
        obj = torch.load(path, weights_only=True)
    if isinstance(obj, torch.Tensor):
        return obj.to(torch.int64).tolist()
    return [int(v) for v in obj]


def load_expert_list(path) -> list:
    with open(path) as f:
        return [int(e) for e in json.load(f)]


def load_wanda_mask(dirpath, t, l, weights_shape=None) -> np.ndarray:
    """Packed mask bits [C, 4C/8] for (t, l) from any supported file in `dirpath`."""
    base = os.path.join(dirpath, f"timestep_{t}_layer_{l}")
    if os.path.exists(base + ".npz"):
        with np.load(base + ".npz", allow_pickle=False) as z:
            return z["bits"]
    if os.path.exists(base + ".pkl"):
        return pack_mask(load_mask_pickle(base + ".pkl"))
    if os.path.exists(base + ".json"):
        if weights_shape is None:
            raise ValueError("JSON index masks need weights_shape")
        idx = np.asarray(json.load(open(base + ".json")), dtype=np.int64).reshape(-1, 2)
        m = np.zeros(tuple(weights_shape[l]), dtype=np.uint8)
        m[idx[:, 0], idx[:, 1]] = 1
        return pack_mask(m)
    raise FileNotFoundError(base + ".{npz,pkl,json}")


def save_wanda_mask(dirpath, t, l, mask):
    os.makedirs(dirpath, exist_ok=True)
    np.savez_compressed(os.path.join(dirpath, f"timestep_{t}_layer_{l}.npz"), bits=pack_mask(mask))
