"""Exception types of the reference's KG path.

``discretekg.py`` raises BoTorch's ``BotorchTensorDimensionError`` and
``UnsupportedError`` (``discretekg.py:15,92-129,175-193,259-273``).  When BoTorch
is importable those very classes are re-exported so ``except`` clauses written
against the reference keep working; otherwise same-named stand-ins are used.
"""

try:  # pragma: no cover - BoTorch is not installed in this image
    from botorch.exceptions import BotorchTensorDimensionError, UnsupportedError  # type: ignore
except Exception:  # noqa: BLE001
    class BotorchTensorDimensionError(Exception):
        """Tensor dimension mismatch (BoTorch stand-in)."""

    class UnsupportedError(Exception):
        """Unsupported configuration (BoTorch stand-in)."""


try:  # pragma: no cover - linear_operator is not installed in this image
    from linear_operator.utils.errors import NotPSDError  # type: ignore
except Exception:  # noqa: BLE001
    class NotPSDError(RuntimeError):
        """Covariance not positive definite after the jitter retries (linear_operator stand-in)."""


class DkgNativeError(RuntimeError):
    """The HIP library is missing, failed to load, or reported a runtime error."""


__all__ = ["BotorchTensorDimensionError", "UnsupportedError", "NotPSDError", "DkgNativeError"]
