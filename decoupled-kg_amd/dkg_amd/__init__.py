"""dkg_amd — MI355X-native Discrete Knowledge Gradient (quasirandom/decoupled-kg hot path).

Drop-in for ``decoupledbo.modules.acquisition.discretekg``; the arithmetic runs
in hand-written HIP kernels for gfx950 behind the C ABI of ``include/dkg.h``.
"""

from .discretekg import (
    DiscreteKnowledgeGradient,
    calculate_discrete_kg,
    calculate_epigraph_indices,
    calculate_epigraph_indices_batched,
    calculate_expected_value_of_piecewise_linear_function,
    calculate_discrete_kg_conditioning_on_single_output,
    clear_state_cache,
    kg_from_lines,
    t_batch_mode_transform,
)
from .errors import BotorchTensorDimensionError, DkgNativeError, UnsupportedError
from .gp_state import DeviceGPState
from .model import ModelListGPState, SingleTaskGPState, from_botorch, from_state_dict
from .utils import is_power_of_2, make_torch_std_grid, sample_simplex

__all__ = [
    "DiscreteKnowledgeGradient",
    "calculate_discrete_kg",
    "calculate_epigraph_indices",
    "calculate_epigraph_indices_batched",
    "calculate_expected_value_of_piecewise_linear_function",
    "calculate_discrete_kg_conditioning_on_single_output",
    "clear_state_cache",
    "kg_from_lines",
    "t_batch_mode_transform",
    "BotorchTensorDimensionError",
    "DkgNativeError",
    "UnsupportedError",
    "DeviceGPState",
    "ModelListGPState",
    "SingleTaskGPState",
    "from_botorch",
    "from_state_dict",
    "is_power_of_2",
    "make_torch_std_grid",
    "sample_simplex",
]
