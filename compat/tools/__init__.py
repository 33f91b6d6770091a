"""Reference import name ``tools`` -> garfield_amd.utils (Context, UserException,
info/warning/error/fatal/trace, pairwise, parse_keyval, TimedContext, flatten, relink,
grads_of, import_directory, cluster_parse)."""
from garfield_amd.utils.flat import flatten, grads_of, relink  # noqa: F401
from garfield_amd.utils.logging import (  # noqa: F401
    Context, UserException, context, error, fatal, info, trace, warning,
)
from garfield_amd.utils.misc import (  # noqa: F401
    ExpandPath, TimedContext, cluster_parse, device_from_tuple, import_directory, make_interface, pairwise,
    parse_keyval, print_args,
)
from garfield_amd.utils.checkpoint import Checkpoints  # noqa: F401
from garfield_amd.utils.flat import flatten_weights, inflate, mapflat, reshape_weights  # noqa: F401,E402
from garfield_amd.utils.profiling import trace_graph  # noqa: F401,E402
from garfield_amd.aggregators.classreg import ClassRegister  # noqa: F401,E402
