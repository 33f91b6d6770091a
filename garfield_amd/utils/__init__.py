"""Utilities: logging contexts, flat-parameter helpers, misc tools, checkpoints."""
from garfield_amd.utils.logging import (  # noqa: F401
    Context, UserException, error, fatal, info, trace, warning,
)
