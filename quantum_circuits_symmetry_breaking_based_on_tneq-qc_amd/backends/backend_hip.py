"""BackendHIP — the 'hip' ComputeBackend (registered via BackendFactory.register_backend,
mirror of tneq_qc/backends/backend_factory.py:91-100).

Contraction entry points (execute_expression, einsum, permute) run on libtneqhip (HIP kernels +
native plans); elementwise bookkeeping ops use torch on the HIP device.  Same constructor
contract as BackendPyTorch (tneq_qc/backends/backend_pytorch.py:16-97): dtype strings
'float32' | 'float64' | 'complex64' | 'complex128' | 'complex', ValueError otherwise.
The native library is loaded at construction: there is no CPU fallback.
"""
from __future__ import annotations

import random
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from .. import _lib
from .backend_interface import BackendInfo, ComputeBackend

_DTYPES = {"float32": "float32", "float64": "float64", "complex64": "complex64",
           "complex128": "complex128", "complex": "complex64"}


class BackendHIP(ComputeBackend):
    def __init__(self, device: Optional[str] = None, dtype: Optional[Any] = None,
                 tensor_type: Optional[str] = None):
        super().__init__(tensor_type=tensor_type)
        import torch
        self.torch = torch
        _lib.lib()  # fail loudly now if libtneqhip.so is missing
        if device is None or device in ("gpu", "hip", "cuda"):
            if not torch.cuda.is_available():
                raise RuntimeError("BackendHIP needs a HIP device (torch.cuda.is_available() is False)")
            device = f"cuda:{torch.cuda.current_device()}"
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError(f"BackendHIP runs on HIP devices only, got device={device!r}")
        self.default_dtype = self._resolve_dtype(dtype)
        self.backend_info = BackendInfo("hip", device=str(self.device),
                                        dtype=str(self.default_dtype).replace("torch.", ""))
        self._einsum_cache: Dict[Tuple, Any] = {}

    def _resolve_dtype(self, dtype):
        torch = self.torch
        if dtype is None:
            return torch.float32
        if isinstance(dtype, str):
            if dtype not in _DTYPES:
                raise ValueError(f"Unsupported dtype string '{dtype}' for BackendHIP. "
                                 f"Supported: {list(_DTYPES.keys())}")
            return getattr(torch, _DTYPES[dtype])
        return dtype

    # ------------------------------------------------------------- contraction surface
    def execute_expression(self, expression, *tensors):
        """backend_interface.py:102-114: the expression is callable on the tensors."""
        return expression(*[self.unwrap_tensor(t) for t in tensors])

    def einsum(self, equation: str, *operands):
        """Any-operand einsum on the HIP engine (plans cached per equation/shapes)."""
        from ..expression import HipContractExpression
        ops = [self.convert_to_tensor(self.unwrap_tensor(o)) for o in operands]
        key = (equation, tuple(tuple(o.shape) for o in ops))
        expr = self._einsum_cache.get(key)
        if expr is None:
            expr = HipContractExpression(equation, *[tuple(o.shape) for o in ops], optimize="greedy")
            self._einsum_cache[key] = expr
        return expr(*ops)

    def permute(self, tensor, dims):
        from ..ops import permute
        return permute(tensor, dims)

    def jit_compile(self, func):
        return func  # plans are compiled natively on first call

    def compute_value_and_grad(self, loss_fn, argnums):
        torch = self.torch

        def value_and_grad_fn(*args):
            idx = list(argnums) if isinstance(argnums, (range, list, tuple)) else [argnums]
            targs = []
            for i, a in enumerate(args):
                a = self.convert_to_tensor(a).detach()
                a.requires_grad_(i in idx)
                targs.append(a)
            loss = loss_fn(*targs)
            lg = loss.real if torch.is_complex(loss) else loss
            if lg.ndim > 0:
                lg = lg.sum()
            grads = torch.autograd.grad(lg, [targs[i] for i in idx])
            out = loss.real.detach() if torch.is_complex(loss) else loss.detach()
            if out.ndim > 0:
                out = out.sum()
            return out, grads

        return value_and_grad_fn

    # ------------------------------------------------------------- tensors
    def convert_to_tensor(self, array):
        torch = self.torch
        if isinstance(array, torch.Tensor):
            t = array
            if t.device != self.device:
                t = t.to(self.device)
            if t.dtype != self.default_dtype:
                t = t.to(self.default_dtype)
            return t
        arr = np.asarray(array)
        return torch.as_tensor(arr, dtype=self.default_dtype).to(self.device)

    def get_backend_name(self) -> str:
        return "hip"

    def init_random_core(self, shape):
        """Orthogonal / unitary init by QR with phase fix (backend_pytorch.py:470-495);
        the QR runs on the host, the core lives on the device."""
        torch = self.torch
        flat = int(np.prod(shape[: len(shape) // 2]))
        cplx = torch.is_complex(torch.zeros(1, dtype=self.default_dtype))
        m = torch.randn((flat, flat), dtype=self.default_dtype)
        q, r = torch.linalg.qr(m)
        d = torch.diag(r)
        if cplx:
            q = q @ torch.diag((d / (d.abs() + 1e-12)).conj())
        else:
            q = q * torch.sign(d).unsqueeze(0)
        return self.wrap_tensor(q.reshape(shape).to(self.device))

    def _get_raw_tensor_type(self):
        return self.torch.Tensor

    def tensor_to_numpy(self, tensor):
        t = self.unwrap_tensor(tensor)
        if not isinstance(t, self.torch.Tensor):
            t = self.torch.as_tensor(t)
        return t.detach().cpu().numpy()

    def set_random_seed(self, seed: int):
        self.torch.manual_seed(seed)
        if self.torch.cuda.is_available():
            self.torch.cuda.manual_seed_all(seed)
        np.random.seed(seed)
        random.seed(seed)

    def reshape(self, tensor, shape):
        return tensor.reshape(shape)

    def eye(self, n: int, dtype=None):
        return self.torch.eye(n, dtype=dtype or self.default_dtype, device=self.device)

    def zeros(self, shape, dtype=None):
        return self.torch.zeros(shape, dtype=dtype or self.default_dtype, device=self.device)

    def ones(self, shape, dtype=None):
        return self.torch.ones(shape, dtype=dtype or self.default_dtype, device=self.device)

    def clone(self, tensor):
        return tensor.clone()

    def unsqueeze(self, tensor, dim):
        return tensor.unsqueeze(dim)

    def expand(self, tensor, *sizes):
        return tensor.expand(*sizes)

    def clamp(self, tensor, min=None, max=None):
        torch = self.torch
        if torch.is_complex(tensor):
            return torch.complex(torch.clamp(tensor.real, min=min, max=max), tensor.imag)
        return torch.clamp(tensor, min=min, max=max)

    def diagonal(self, tensor, dim1=-2, dim2=-1):
        return self.torch.diagonal(tensor, dim1=dim1, dim2=dim2)

    def sum(self, tensor, dim=None, keepdim=False):
        return self.torch.sum(tensor, dim=dim, keepdim=keepdim) if dim is not None else self.torch.sum(tensor)

    def multinomial(self, probs, num_samples):
        return self.torch.multinomial(probs, num_samples=num_samples)

    def arange(self, *args, dtype=None):
        return self.torch.arange(*args, dtype=dtype or self.torch.long, device=self.device)

    def stack(self, tensors, dim=0):
        return self.torch.stack(tensors, dim=dim)

    def log(self, tensor):
        return self.torch.log(tensor)

    def mean(self, tensor, dim=None, keepdim=False):
        return self.torch.mean(tensor, dim=dim, keepdim=keepdim) if dim is not None else self.torch.mean(tensor)

    def squeeze(self, tensor, dim=None):
        return tensor.squeeze() if dim is None else tensor.squeeze(dim)

    def detach(self, tensor):
        return tensor.detach() if hasattr(tensor, "detach") else tensor

    def exp(self, tensor):
        return self.torch.exp(tensor)

    def sqrt(self, tensor):
        return self.torch.sqrt(tensor)

    def square(self, tensor):
        return self.torch.square(tensor)

    def lgamma(self, tensor):
        return self.torch.lgamma(tensor)

    def ones_like(self, tensor):
        return self.torch.ones_like(tensor)

    def linspace(self, start, end, steps, dtype=None):
        return self.torch.linspace(start, end, steps, dtype=dtype or self.default_dtype, device=self.device)

    def cumsum(self, tensor, dim, dtype=None):
        return self.torch.cumsum(tensor, dim=dim, dtype=dtype)

    def rand(self, size, dtype=None):
        return self.torch.rand(size, dtype=dtype or self.default_dtype, device=self.device)

    def real(self, tensor):
        return self.torch.real(tensor)

    def gather(self, input, dim, index):
        return self.torch.gather(input, dim, index)

    def is_complex(self, tensor) -> bool:
        return self.torch.is_complex(self.unwrap_tensor(tensor))

    def abs_square(self, tensor):
        """Born rule |x|^2 for complex, identity for real (backend_pytorch.py:655-660)."""
        if self.torch.is_complex(tensor):
            return tensor.real * tensor.real + tensor.imag * tensor.imag
        return tensor

    # ------------------------------------------------------------- optimizer (training path)
    def optimizer_update(self, params: List[Any], grads: List[Any], state: Dict[str, Any],
                         method: str, hyperparams: Dict[str, Any]):
        """sgd / momentum / adam / sgdg steps with the reference's hyper-parameter names
        (backend_pytorch.py:200-468); TNTensor params are updated in their unscaled frame."""
        from ..core.tn_tensor import TNTensor
        torch = self.torch
        lr = hyperparams.get("learning_rate", 0.01)
        with torch.no_grad():
            raw, info = [], []
            for p in params:
                if isinstance(p, TNTensor):
                    raw.append(p.tensor * p.scale)
                    info.append(p.scale)
                else:
                    raw.append(p)
                    info.append(None)
            grads = [g / s if s is not None else g for g, s in zip(grads, info)]
            if method == "sgd":
                new = [p - lr * g for p, g in zip(raw, grads)]
            elif method == "momentum":
                buf = state.setdefault("momentum_buffer", [torch.zeros_like(p) for p in raw])
                new = []
                for i, (p, g) in enumerate(zip(raw, grads)):
                    buf[i] = 0.9 * buf[i] + lr * g
                    new.append(p - buf[i])
            elif method == "adam":
                b1, b2 = hyperparams.get("beta1", 0.9), hyperparams.get("beta2", 0.999)
                eps, it = hyperparams.get("epsilon", 1e-8), hyperparams.get("iter", 0)
                m = state.setdefault("m", [torch.zeros_like(p) for p in raw])
                v = state.setdefault("v", [torch.zeros_like(p) for p in raw])
                new = []
                for i, (p, g) in enumerate(zip(raw, grads)):
                    m[i] = b1 * m[i] + (1 - b1) * g
                    v[i] = b2 * v[i] + (1 - b2) * (g * g.conj()).real
                    mh = m[i] / (1 - b1 ** (it + 1))
                    vh = v[i] / (1 - b2 ** (it + 1))
                    new.append(p - lr * mh / (torch.sqrt(vh) + eps))
            elif method == "sgdg":
                new = self._sgdg(raw, grads, state, hyperparams)
            else:
                raise ValueError(f"Unknown optimization method: {method}")
            out = []
            for n, s in zip(new, info):
                if s is not None:
                    t = TNTensor(n / s, s)
                    t.tensor.requires_grad_(True)
                    out.append(t)
                else:
                    n.requires_grad_(True)
                    out.append(n)
            return out, state

    def _sgdg(self, params, grads, state, hp):
        """Stiefel SGD with the Cayley transform (backend_pytorch.py:349-468)."""
        torch = self.torch
        lr, mom, stiefel = hp.get("learning_rate", 0.01), hp.get("momentum", 0.0), hp.get("stiefel", True)
        bufs = state.setdefault("momentum_buffer", [None] * len(params))
        out = []
        for i, (p, g) in enumerate(zip(params, grads)):
            shp = p.shape
            if len(shp) > 2:
                fd = int(np.prod(shp[: len(shp) // 2]))
                p2, g2 = p.reshape(fd, -1), g.reshape(fd, -1)
            else:
                p2, g2 = p, g
            cplx = torch.is_complex(p2)
            nrm = torch.norm(p2, p=2, dim=1, keepdim=True)
            X = p2 / (nrm + 1e-8)
            if stiefel and X.shape[0] <= X.shape[1]:
                if bufs[i] is None:
                    bufs[i] = torch.zeros(g2.T.shape, dtype=g2.dtype, device=p.device)
                gT = g2.conj().T if cplx else g2.T
                V = mom * bufs[i] - gT
                MX = V @ X
                XMX = X @ MX
                XH = X.conj().T if cplx else X.T
                W_hat = MX - 0.5 * (XH @ XMX)
                W = W_hat - (W_hat.conj().T if cplx else W_hat.T)
                t = 0.5 * 2 / (torch.abs(W).sum(dim=0).max() + 1e-8)
                alpha = min(float(t), lr)
                I = torch.eye(W.shape[0], dtype=W.dtype, device=W.device)
                Y = torch.linalg.solve(I - (alpha / 2) * W, (I + (alpha / 2) * W) @ (XH if cplx else X.T))
                pn = Y.conj().T if cplx else Y.T
                out.append(pn.reshape(shp))
                bufs[i] = W @ XH
            else:
                out.append(p - lr * g)
        return out
