"""gpfit — MI355X-native GP-fit hot path (HIP kernels behind a C-ABI).

Internal package of the drop-in modules that sit next to it
(GP_func.py, find_len_scales.py, ...). See DESIGN.md.
"""
from ._lib import (Comm, Context, GPFitError, build_info, default_comm, default_context, load_library,  # noqa: F401
                   plan_check)
