"""aclswarm_amd -- MI355X-native batched engine for aclswarm's per-vehicle
decision loop (CBAA auction + distributed control + safety + ADMM gains).

The compute lives in the HIP library aclswarm_amd/lib/libaclswarm_amd.so
behind the C ABI declared in include/aclswarm_amd.h. There is no CPU fallback.
"""
from . import _lib  # noqa: F401
from ._lib import (FLAG_AGREE, FLAG_BAD_INPUT, FLAG_CA_ACTIVE, FLAG_CHANGED,  # noqa: F401
                   FLAG_NONFINITE, FLAG_VALID, STATUS_DTYPE, lib)

__all__ = ["lib", "STATUS_DTYPE"]
