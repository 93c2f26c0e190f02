"""Discrete multi-objective knowledge gradient on MI355X — drop-in host mirror.

Same surface as the reference's
``decoupledbo.modules.acquisition.discretekg`` (``discretekg.py:25-338``):

* ``DiscreteKnowledgeGradient(model, x_discretisation, scalarisation_weights=None,
  target_output_ix=None)`` with ``create_with_sobol_sample``, ``set_X_pending``
  and ``forward(X[*batch, 1, d]) -> [*batch]`` (``:33-159``);
* ``calculate_discrete_kg`` (``:162-235``) and
  ``calculate_discrete_kg_conditioning_on_single_output`` (``:238-338``);
* ``calculate_epigraph_indices`` (``:341-412``, the reference's walk exactly) and
  ``calculate_expected_value_of_piecewise_linear_function`` (``:415-452``), device-backed;
* ``kg_from_lines`` — the epigraph + expectation stage
  (``calculate_epigraph_indices`` + ``calculate_expected_value_of_piecewise_linear_function``
  + ``- max(intercepts)``, ``:225-233, 341-452``) batched on the device.

The fitted GP state lives in HBM (``gp_state.DeviceGPState``); every forward
is three HIP kernel launches through the C ABI (``include/dkg.h``).  There is
no CPU fallback: without the HIP library or a ROCm device these raise.
"""

from __future__ import annotations

import math
from functools import wraps
from typing import Optional

import torch
from torch import Tensor

from . import _lib
from .errors import BotorchTensorDimensionError, UnsupportedError
from .gp_state import DeviceGPState, current_stream_ptr
from .model import ModelListGPState, SingleTaskGPState, from_botorch

try:  # pragma: no cover - BoTorch is not installed in this image
    from botorch.acquisition import AcquisitionFunction as _Base  # type: ignore

    _HAVE_BOTORCH = True
except Exception:  # noqa: BLE001
    _Base = torch.nn.Module
    _HAVE_BOTORCH = False


def t_batch_mode_transform(expected_q: Optional[int] = None):
    """BoTorch ``t_batch_mode_transform`` (as used at ``discretekg.py:131``)."""

    def decorator(method):
        @wraps(method)
        def decorated(acqf, X, *args, **kwargs):
            if not isinstance(X, Tensor):
                return method(acqf, X, *args, **kwargs)
            if X.dim() < 2:
                raise ValueError(
                    f"{type(acqf).__name__} requires X to have at least 2 dimensions,"
                    f" but received X with only {X.dim()} dimensions.")
            if expected_q is not None and X.shape[-2] != expected_q:
                raise AssertionError(
                    f"Expected X to be `batch_shape x q={expected_q} x d`, but got X with shape {X.shape}.")
            X = X if X.dim() > 2 else X.unsqueeze(0)
            return method(acqf, X, *args, **kwargs)

        return decorated

    return decorator


def _as_model_state(model) -> ModelListGPState:
    if isinstance(model, ModelListGPState):
        return model
    if isinstance(model, SingleTaskGPState):
        return ModelListGPState(model)
    return from_botorch(model)


_BY_VALUE_NUMEL = 64  # tensors this small are fingerprinted by value as well


_VIEWS: dict = {}  # id -> (tensor, data_ptr, numpy view of its memory): the by-value read without new tensors


def _small_values(t):
    """(data pointer, the bytes of the values) of a small CPU tensor, read through a cached numpy view of its
    memory (~0.5 us against ~6 us for detach().tolist() per call: this runs on every forward)."""
    p = t.data_ptr()
    e = _VIEWS.get(id(t))
    if e is None or e[0] is not t or e[1] != p:
        if len(_VIEWS) > 256:
            _VIEWS.clear()
        e = (t, p, t.detach().numpy())
        _VIEWS[id(t)] = e
    return (p, e[2].tobytes())


def _fingerprint(obj):
    """What the fitted state of ``model`` is made of, cheaply: every tensor by (identity, in-place
    version counter), every other field by value.  The reference reads the model live at every
    forward (``model.posterior``, discretekg.py:182-185, 275-284); the device state is rebuilt
    whenever this changes (a refit, new training data, an in-place edit)."""
    if isinstance(obj, torch.Tensor):
        if obj.is_cpu and obj.numel() <= _BY_VALUE_NUMEL:
            # hyperparameters (lengthscales, outputscale, noise, constant mean, Standardize buffers): by value,
            # since gpytorch's initialize() and constraint setters write them through .data, which does not
            # bump the version counter.  Device-resident ones are fingerprinted by identity and version only
            # (a by-value read would synchronise the device on every forward): after editing the
            # hyperparameters of a model that lives on the GPU through .data / initialize(), call
            # clear_state_cache() and DiscreteKnowledgeGradient.invalidate()
            return (id(obj), obj._version) + _small_values(obj)
        return (id(obj), obj._version)
    if isinstance(obj, ModelListGPState):  # flat, no recursion or generator: this runs on every forward
        parts = []
        for m in obj.models:
            tx, ty, ls = m.train_x, m.train_y, m.lengthscale
            # (SingleTaskGPState keeps its tensors on the host: __post_init__; a device lengthscale assigned later
            # is fingerprinted by identity and version only, as _fingerprint does)
            lsv = _small_values(ls) if ls.is_cpu else None
            parts.append((id(tx), tx._version, id(ty), ty._version, id(ls), ls._version, lsv, m.outputscale, m.noise,
                          m.mean_constant, m.kernel, m.nu, m.y_mean, m.y_std))
        return tuple(parts)
    if isinstance(obj, SingleTaskGPState):
        return _fingerprint(ModelListGPState(obj))
    if isinstance(obj, torch.nn.Module):  # a BoTorch model: parameters, buffers and training data
        parts = [_fingerprint(t) for t in obj.parameters()] + [_fingerprint(t) for t in obj.buffers()]
        for sub in getattr(obj, "models", None) or [obj]:
            parts += [_fingerprint(t) for t in getattr(sub, "train_inputs", ()) or ()]
            tt = getattr(sub, "train_targets", None)
            if tt is not None:
                parts.append(_fingerprint(tt))
        return tuple(parts)
    return id(obj)


def _weights_fingerprint(w):
    """The scalarisation weights by identity and version counter, and by value when they are a small host
    tensor (an edit through ``.data`` does not bump the version counter).  A device-resident weights tensor
    edited through ``.data`` is not seen (reading it back would cost a device synchronisation per forward):
    assign a new tensor instead."""
    if w.is_cpu and w.numel() <= 4096:
        return (id(w), w._version) + _small_values(w)
    return (id(w), w._version)


# Device states of recently used (model, discretisation) pairs.  The reference builds one acquisition
# per output on the same fitted model and grid (acquisition_optimisation_strategy.py:209-216, one
# DiscreteKnowledgeGradient per obj_idx_new), and every one reads the same posterior caches: they share
# one DeviceGPState instead of each repeating the Cholesky, the inverse and the cross products.  An entry
# holds its model's tensors alive, so no live tensor can take over an id in its fingerprint.
_STATE_CACHE: list = []
_STATE_CACHE_SIZE = 4


def clear_state_cache() -> None:
    """Drop every shared device state (e.g. between BO iterations, after a refit): the next acquisition
    rebuilds its caches, and the device memory of the dropped states is released with their last user."""
    _STATE_CACHE.clear()


def shared_state(state: ModelListGPState, fp, x_discretisation: Tensor, device, owner=None) -> DeviceGPState:
    """The cached DeviceGPState of (model fingerprint ``fp``, discretisation values, device), or a new one.
    ``owner`` (the caller's model object) is kept alive with the entry, with its fingerprinted tensors."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    D = x_discretisation.detach()
    for i, (efp, eD, edev, est, _) in enumerate(_STATE_CACHE):
        if efp == fp and edev == dev and eD.shape == D.shape and eD.dtype == D.dtype and torch.equal(eD, D.to(eD.device)):
            _STATE_CACHE.insert(0, _STATE_CACHE.pop(i))
            return est
    st = DeviceGPState(state, x_discretisation, dev)
    _STATE_CACHE.insert(0, (fp, D.clone(), dev, st, owner))
    del _STATE_CACHE[_STATE_CACHE_SIZE:]
    return st


class _ForwardFn(torch.autograd.Function):
    """Device forward; when X requires grad the same C call also returns
    dKG(x_b)/dx_b (dkg_plan_forward_grad), and backward scales it by the
    incoming gradient.  KG(x_b) depends on x_b only, so the Jacobian is
    block-diagonal and this is the exact vector-Jacobian product."""

    @staticmethod
    def forward(ctx, X, acq):
        if ctx.needs_input_grad[0]:
            kg, dkg = acq._plan_for(X.shape[0], grad=True).forward_grad(X)
            ctx.save_for_backward(dkg)
            return kg
        return acq._plan_for(X.shape[0]).forward(X)

    @staticmethod
    def backward(ctx, grad):
        (dkg,) = ctx.saved_tensors
        return grad.to(dkg)[:, None] * dkg, None


class _HostForwardFn(torch.autograd.Function):
    """``forward`` of host candidates (what ``optimize_acqf`` passes: a host X [*batch, 1, d] with
    ``requires_grad``): one device round trip per call -- with a gradient, the candidates in the first
    kernel's arguments and [KG | dKG/dx] written by the envelope kernel into pinned memory
    (``ForwardPlan.forward_grad_host``); without, a pinned copy each way -- and a host-side backward.
    The reshapes and the dtype round trip happen inside, so the autograd graph is this one node.  The
    same kernels as ``_ForwardFn``, so the same bits."""

    @staticmethod
    def forward(ctx, X, acq):
        d = X.shape[-1]
        batch = X.shape[:-2]
        xs = X  # (inside an autograd.Function's forward: its data pointer is read)
        if xs.dtype is not torch.double or not xs.is_contiguous():
            xs = xs.detach().to(torch.double).contiguous()
        B = xs.numel() // d
        if ctx.needs_input_grad[0]:
            plan = acq._plan_grad
            if plan is None or plan.max_B < B:
                plan = acq._plan_for(B, grad=True)
            kg, dkg = plan.forward_grad_host_shaped(xs, B, batch, X.shape)
            ctx.save_for_backward(dkg)
            ctx.xdtype = X.dtype
            return kg if X.dtype == torch.double else kg.to(X.dtype)
        kg = acq._plan_for(B).forward_host(xs.reshape(B, d))
        return kg.to(X.dtype).reshape(batch)

    @staticmethod
    def backward(ctx, grad):
        (dkg,) = ctx.saved_tensors  # shaped as X: [*batch, 1, d]
        g = grad.to(dkg) if grad.dtype != dkg.dtype else grad
        out = g.reshape(g.shape + (1, 1)) * dkg
        return (out if ctx.xdtype == torch.double else out.to(ctx.xdtype)), None


class DiscreteKnowledgeGradient(_Base):
    """Discrete knowledge gradient (C-MOKG), linear scalarisations only."""

    @classmethod
    def create_with_sobol_sample(cls, model, bounds: Tensor, num_discrete_points: int,
                                 scalarisation_weights: Optional[Tensor] = None,
                                 target_output_ix: Optional[int] = None):
        """Sobol discretisation (``discretekg.py:33-60``): ``draw_sobol_samples(bounds, N, q=1)``,
        whose scrambling seed is drawn from torch's global RNG, so ``torch.manual_seed`` fixes it."""
        from .optim import draw_sobol_samples

        x_disc = draw_sobol_samples(bounds, num_discrete_points, q=1).squeeze(1).to(bounds)
        return cls(model, x_disc, scalarisation_weights, target_output_ix)

    def __init__(self, model, x_discretisation: Tensor, scalarisation_weights: Optional[Tensor] = None,
                 target_output_ix: Optional[int] = None, device=None, precision: str = "fp64"):
        if _HAVE_BOTORCH:  # pragma: no cover
            super().__init__(model=model)
        else:
            super().__init__()
            self.model = model
        state = _as_model_state(model)
        if x_discretisation.dim() != 2:
            raise BotorchTensorDimensionError(
                f"Expected 'x_discretisation' to have two dimensions. "
                f"Got {x_discretisation.dim()=}.")
        if scalarisation_weights is None:
            if state.num_outputs != 1:
                raise UnsupportedError("Models with more than one output must specify 'scalarisation_weights'.")
            scalarisation_weights = torch.tensor([[1.0]]).to(x_discretisation)
        if scalarisation_weights.dim() != 2:
            raise BotorchTensorDimensionError(
                f"Expected 'scalarisation_weights' to have two dimensions: The first "
                f"indexing different scalarisations to be averaged over and the second "
                f"indexing coordinates of the objective space. "
                f"Got {scalarisation_weights.dim()=}")
        if scalarisation_weights.shape[-1] != state.num_outputs:
            raise BotorchTensorDimensionError(
                f"Expected the last dimension of 'scalarisation_weights' to have one "
                f"element per objective. Got {scalarisation_weights.shape[-1]=} != "
                f"{state.num_outputs}=model.num_outputs.")
        if precision not in ("fp64", "fp32"):
            raise ValueError(f"precision must be 'fp64' (the reference's) or 'fp32', got {precision!r}")
        # "fp32": the two contractions of the forward in fp32 MFMA (include/dkg.h DKG_PLAN_F32;
        # BASELINE configs[4]); not a reference mode, forward only
        self.precision = precision
        self.x_discretisation = x_discretisation
        self.scalarisation_weights = scalarisation_weights
        self.target_output_ix = target_output_ix
        # the reference indexes the outputs with it (posteriors[obj_idx_new], weights[..., obj_idx_new],
        # discretekg.py:301-321): a negative index counts from the end, one out of range raises
        # IndexError when the KG is evaluated
        self._target = None
        self._target_error = None
        if target_output_ix is not None:
            t = int(target_output_ix)
            if -state.num_outputs <= t < state.num_outputs:
                self._target = t % state.num_outputs
            else:
                self._target_error = IndexError("list index out of range")
        self._device = device
        self._fp = _fingerprint(model)
        self._state = shared_state(state, self._fp, x_discretisation, device, owner=model)
        self._wfp = _weights_fingerprint(scalarisation_weights)
        self._W = scalarisation_weights.detach().to(self._state.device, torch.double, copy=True).contiguous()
        self._plan = None
        self._plan_grad = None

    def _refresh(self):
        """Rebuild the device state if the model changed since it was read (see _fingerprint), and the plans
        if the scalarisation weights did: the reference reads both live at every forward (discretekg.py:
        131-159, 182-185).  The plans hold a snapshot of the weights (their intercept caches are derived from
        it), so an in-place edit of ``scalarisation_weights`` or a new tensor assigned to it is seen here."""
        fp = _fingerprint(self.model)
        if fp != self._fp:
            self._state = shared_state(_as_model_state(self.model), fp, self.x_discretisation, self._device,
                                       owner=self.model)
            self._plan = None
            self._plan_grad = None
            self._fp = fp
        wfp = _weights_fingerprint(self.scalarisation_weights)
        if wfp != self._wfp:
            w = self.scalarisation_weights
            if w.dim() != 2 or w.shape[-1] != self._W.shape[-1]:
                raise BotorchTensorDimensionError(
                    f"Expected 'scalarisation_weights' to stay S x {self._W.shape[-1]}. Got {tuple(w.shape)}.")
            self._W = w.detach().to(self._state.device, torch.double, copy=True).contiguous()
            self._plan = None
            self._plan_grad = None
            self._wfp = wfp

    def invalidate(self) -> None:
        """Re-read the model at the next forward whatever its fingerprint says (a device-resident model whose
        hyperparameters were edited through ``.data``, which the fingerprint cannot see without a device
        synchronisation per forward).  Also drops the shared device state built from the old values."""
        clear_state_cache()
        self._fp = None

    def _plan_for(self, B: int, grad: bool = False):
        """The forward plan (with gradient buffers when ``grad``), grown (powers of two) to hold B candidates."""
        cur = self._plan_grad if grad else self._plan
        if cur is None or cur.max_B < B:
            cap = 1
            while cap < B:
                cap *= 2
            if grad and self.precision == "fp32":
                raise UnsupportedError("precision='fp32' is forward only; use precision='fp64' for gradients")
            if self._target_error is not None:
                raise self._target_error
            cur = self._state.plan(self._W, self._target, max(cap, 16), grad=grad, f32=self.precision == "fp32")
            if grad:
                self._plan_grad = cur
            else:
                self._plan = cur
        return cur

    def set_X_pending(self, X_pending: Optional[Tensor] = None) -> None:
        raise UnsupportedError(f"{type(self).__name__} does not account for X_pending yet.")

    @t_batch_mode_transform(expected_q=1)
    def forward(self, X: Tensor) -> Tensor:
        batch_shape, d = X.shape[:-2], X.shape[-1]
        if d != self.x_discretisation.shape[-1]:
            raise RuntimeError(
                f"Expected X to have last dimension matching 'self.x_discretisation'. "
                f"Got {X.shape[-1]=}, {self.x_discretisation.shape[-1]=}.")
        self._refresh()
        if X.device.type == "cpu":  # the host route: one round trip (and a host backward)
            return _HostForwardFn.apply(X, self)
        flat = X.reshape(-1, d)
        Xd = flat.to(self._state.device, torch.double)
        kg = _ForwardFn.apply(Xd, self)
        return kg.to(device=X.device, dtype=X.dtype).reshape(batch_shape)

    def value_and_grad_host(self, X: Tensor):
        """KG and dKG/dX for host candidates X (``[*batch, 1, d]`` or ``[B, d]``), as host fp64 tensors of
        shapes ``batch`` and ``X.shape``: what one L-BFGS-B evaluation of ``optimize_acqf`` needs back
        (``bo_loop.py:127-129``, ``batch_limit = 1``).  The same values and gradient as ``forward`` +
        autograd, with one device round trip and no autograd graph: up to 64 candidate coordinates travel in
        the first kernel's arguments and the envelope kernel writes [KG | dKG/dX] into pinned host memory
        (``ForwardPlan.forward_grad_host``; larger batches: one pinned copy each way)."""
        d = self.x_discretisation.shape[-1]
        if X.shape[-1] != d:
            raise RuntimeError(
                f"Expected X to have last dimension matching 'self.x_discretisation'. "
                f"Got {X.shape[-1]=}, {self.x_discretisation.shape[-1]=}.")
        if X.dim() > 2 and X.shape[-2] != 1:
            raise ValueError(f"Expected X to be `batch_shape x q=1 x d`, but got X with shape {tuple(X.shape)}.")
        self._refresh()
        xs = X  # (its data pointer is read, nothing is recorded for autograd)
        if xs.dtype is not torch.double or not xs.is_cpu or not xs.is_contiguous():
            xs = xs.detach().to("cpu", torch.double).contiguous()
        B = xs.numel() // d
        plan = self._plan_grad
        if plan is None or plan.max_B < B:
            plan = self._plan_for(B, grad=True)
        batch = X.shape[:-2] if X.dim() > 2 else X.shape[:-1]
        return plan.forward_grad_host_shaped(xs, B, batch, X.shape)

    def forward_pairs(self, X: Tensor) -> Tensor:
        """KG per (candidate, scalarisation): [B, S] (the per-``j`` values of ``:200-233``)."""
        self._refresh()
        flat = X.reshape(-1, X.shape[-1])
        pairs = torch.empty(flat.shape[0], self._W.shape[0], dtype=torch.double, device=self._state.device)
        self._plan_for(flat.shape[0]).forward(flat, kg_pairs=pairs)
        return pairs


def _check_weights(w: Tensor) -> None:
    if w.dim() != 2:
        raise BotorchTensorDimensionError(
            "Expected 'scalarisation_weights' to have two dimensions: The first "
            "indexing different scalarisations to be averaged over and the second "
            "indexing coordinates of the objective space.")


def calculate_discrete_kg(model, xnew: Tensor, discretisation: Tensor, scalarisation_weights: Tensor) -> Tensor:
    """KG at one candidate, all outputs observed (``discretekg.py:162-235``)."""
    _check_weights(scalarisation_weights)
    acq = DiscreteKnowledgeGradient(model, discretisation, scalarisation_weights)
    return acq(xnew.reshape(1, 1, -1)).reshape(())


def calculate_discrete_kg_conditioning_on_single_output(model, xnew: Tensor, obj_idx_new: int,
                                                        discretisation: Tensor,
                                                        scalarisation_weights: Tensor) -> Tensor:
    """KG at one candidate observing output ``obj_idx_new`` only (``discretekg.py:238-338``)."""
    _check_weights(scalarisation_weights)
    state = _as_model_state(model)
    if not isinstance(state, ModelListGPState):
        raise UnsupportedError(f"Input 'model' must be a 'ModelListGP'. Got {type(model)=}.")
    acq = DiscreteKnowledgeGradient(state, discretisation, scalarisation_weights, target_output_ix=obj_idx_new)
    return acq(xnew.reshape(1, 1, -1)).reshape(())


def _verify_intercepts_and_slopes(intercepts: Tensor, slopes: Tensor) -> None:
    """The reference's checks and messages (``discretekg.py:455-470``)."""
    if intercepts.dim() != 1 or slopes.dim() != 1:
        raise BotorchTensorDimensionError(
            f"Expected 'intercepts' and 'slopes' to both be one-dimensional tensors. "
            f"Got {intercepts.dim()=} and {slopes.dim()=}.")
    if intercepts.shape != slopes.shape:
        raise BotorchTensorDimensionError(
            f"Expected 'intercepts' and 'slopes' to have the same shape. "
            f"Got {intercepts.shape=} and {slopes.shape=}.")
    if intercepts.shape[-1] == 0:
        raise ValueError(f"Expected inputs to specify at least one line. Got {intercepts.shape[-1]=}.")


def _device_of(t: Tensor) -> torch.device:
    return t.device if t.is_cuda else torch.device("cuda", torch.cuda.current_device())


def calculate_epigraph_indices_batched(intercepts: Tensor, slopes: Tensor):
    """The reference walk (``calculate_epigraph_indices``, ``discretekg.py:341-412``) for a batch
    of line sets ``[..., L]``, on the device (``dkg_epigraph``).

    Returns ``(indices [..., L] int64, intersections [..., L-1], counts [...] int32)``: set p's
    envelope is ``indices[p, :counts[p]]`` with breakpoints ``intersections[p, :counts[p]-1]``;
    entries past the count are -1 / NaN.  Computed in fp64.
    """
    if intercepts.shape != slopes.shape:
        raise BotorchTensorDimensionError(
            f"Expected 'intercepts' and 'slopes' to have the same shape. "
            f"Got {intercepts.shape=} and {slopes.shape=}.")
    if intercepts.dim() < 1:
        raise BotorchTensorDimensionError("Expected 'intercepts' and 'slopes' to have at least one dimension.")
    L = intercepts.shape[-1]
    if L == 0:
        raise ValueError(f"Expected inputs to specify at least one line. Got intercepts.shape[-1]={L}.")
    lib = _lib.load()
    dev = _device_of(intercepts)
    a = intercepts.detach().to(dev, torch.double).reshape(-1, L).contiguous()
    b = slopes.detach().to(dev, torch.double).reshape(-1, L).contiguous()
    P = a.shape[0]
    idx = torch.full((P, L), -1, dtype=torch.int64, device=dev)
    xs = torch.full((P, max(L - 1, 1)), float("nan"), dtype=torch.double, device=dev)
    cnt = torch.zeros(P, dtype=torch.int32, device=dev)
    _lib.check(lib.dkg_epigraph(_lib.ptr(a), _lib.ptr(b), P, L, L, _lib.ptr(idx), _lib.ptr(xs), _lib.ptr(cnt),
                                current_stream_ptr(dev)), "dkg_epigraph")
    shape = intercepts.shape[:-1]
    return idx.reshape(*shape, L), xs[:, : L - 1].reshape(*shape, L - 1), cnt.reshape(shape)


def calculate_epigraph_indices(intercepts: Tensor, slopes: Tensor):
    """Upper envelope of the lines ``a_k + b_k z`` (``discretekg.py:341-412``), on the device.

    Same results as the reference: the line indices left to right and the intersections
    between successive ones, the same IEEE values (``include/dkg.h`` ``dkg_epigraph``).  The
    intersections are recomputed from the returned indices with the reference's expression,
    so they carry the reference's autograd graph w.r.t. ``intercepts`` / ``slopes``.
    """
    _verify_intercepts_and_slopes(intercepts, slopes)
    idx, xs, cnt = calculate_epigraph_indices_batched(intercepts.reshape(1, -1), slopes.reshape(1, -1))
    m = int(cnt[0])
    indices = idx[0, :m].to(intercepts.device)
    if m < 2:
        return indices, torch.tensor([], dtype=intercepts.dtype, device=intercepts.device)
    if intercepts.requires_grad or slopes.requires_grad:
        i0, i1 = indices[:-1], indices[1:]
        inter = -(intercepts[i0] - intercepts[i1]) / (slopes[i0] - slopes[i1])  # discretekg.py:394
    else:
        inter = xs[0, : m - 1].to(device=intercepts.device, dtype=intercepts.dtype)
    return indices, inter


class _PiecewiseExpectation(torch.autograd.Function):
    """E[f(Z)] on the device; backward by the closed form of the reference expression
    (d/da_j = dPhi_j, d/db_j = -dphi_j, d/dc_k = phi(c_k) (a_{k-1} - a_k + c_k (b_{k-1} - b_k)))."""

    @staticmethod
    def forward(ctx, a, b, c):
        lib = _lib.load()
        dev = _device_of(a)
        m = a.shape[0]
        ad = a.detach().to(dev, torch.double).contiguous()
        bd = b.detach().to(dev, torch.double).contiguous()
        cd = c.detach().to(dev, torch.double).contiguous()
        out = torch.empty(1, dtype=torch.double, device=dev)
        _lib.check(lib.dkg_pwl_expectation(_lib.ptr(ad), _lib.ptr(bd), _lib.ptr(cd) if m > 1 else 0, 1, m,
                                           _lib.ptr(out), current_stream_ptr(dev)), "dkg_pwl_expectation")
        ctx.save_for_backward(a, b, c)
        return out.reshape(()).to(device=a.device, dtype=a.dtype)

    @staticmethod
    def backward(ctx, g):
        a, b, c = ctx.saved_tensors
        inf = torch.full((1,), float("inf"), dtype=c.dtype, device=c.device)
        z = torch.cat([-inf, c, inf])
        pdf = torch.where(torch.isinf(z), torch.zeros_like(z), torch.exp(-0.5 * z * z) / math.sqrt(2 * math.pi))
        cdf = 0.5 * (1 + torch.erf(z / math.sqrt(2)))
        ga = (cdf[1:] - cdf[:-1]) * g
        gb = -(pdf[1:] - pdf[:-1]) * g
        gc = pdf[1:-1] * ((a[:-1] - a[1:]) + c * (b[:-1] - b[1:])) * g
        return ga, gb, gc


def calculate_expected_value_of_piecewise_linear_function(intercepts: Tensor, slopes: Tensor, boundaries: Tensor):
    """E[f(Z)] for Z ~ N(0, 1) and piecewise-linear f (``discretekg.py:415-452``), on the device
    (``dkg_pwl_expectation``, the reference's formula); differentiable."""
    _verify_intercepts_and_slopes(intercepts, slopes)
    if boundaries.shape != (len(intercepts) - 1,):
        raise BotorchTensorDimensionError(
            f"Expected 'boundaries' to be a one-dimensional tensor with "
            f"{len(intercepts)} elements. Got {boundaries.shape=}.")
    return _PiecewiseExpectation.apply(intercepts, slopes, boundaries)


def kg_from_lines(intercepts: Tensor, slopes: Tensor, return_hull_size: bool = False):
    """E[max_k (a_k + b_k Z)] - max_k a_k per set of lines, on the device.

    ``intercepts``/``slopes``: [..., L] (same shape).  Batched form of the
    reference's epigraph + expectation + baseline (``discretekg.py:225-233``).
    """
    if intercepts.shape != slopes.shape:
        raise BotorchTensorDimensionError(
            f"Expected 'intercepts' and 'slopes' to have the same shape. "
            f"Got {intercepts.shape=} and {slopes.shape=}.")
    if intercepts.dim() < 1:
        raise BotorchTensorDimensionError("Expected 'intercepts' and 'slopes' to have at least one dimension.")
    L = intercepts.shape[-1]
    if L == 0:
        raise ValueError(f"Expected inputs to specify at least one line. Got intercepts.shape[-1]={L}.")
    lib = _lib.load()
    dev = _device_of(intercepts)
    a = intercepts.detach().to(dev, torch.double).reshape(-1, L).contiguous()
    b = slopes.detach().to(dev, torch.double).reshape(-1, L).contiguous()
    P = a.shape[0]
    kg = torch.empty(P, dtype=torch.double, device=dev)
    hull = torch.empty(P, dtype=torch.int32, device=dev) if return_hull_size else None
    _lib.check(lib.dkg_lines_kg(_lib.ptr(a), _lib.ptr(b), P, L, _lib.ptr(kg), _lib.ptr(hull),
                                current_stream_ptr(dev)), "dkg_lines_kg")
    out = kg.reshape(intercepts.shape[:-1]).to(intercepts.device)
    if return_hull_size:
        return out, hull.reshape(intercepts.shape[:-1]).to(intercepts.device)
    return out
