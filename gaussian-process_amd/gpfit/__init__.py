"""gpfit — MI355X-native GP-fit hot path (HIP kernels behind a C-ABI).

Internal package of the drop-in modules that sit next to it
(GP_func.py, find_len_scales.py, ...). See DESIGN.md.
"""
from ._lib import Context, GPFitError, build_info, default_context, load_library, plan_check  # noqa: F401
