"""Robust aggregation operators (native CPU / gfx950 HIP) and their fp64 references."""
from garfield_amd.ops import reference  # noqa: F401
from garfield_amd.ops.gar import (  # noqa: F401
    MAX_ROWS, RULES, aggregate, aksel, aksel_weights, average, average_nan, averaged_median, brute,
    brute_weights, bulyan, bulyan_weights, combine, condense, gram, krum, krum_weights, median,
    pairwise_distances, prepare, trimmed_mean,
)
