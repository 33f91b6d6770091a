from garfield_amd.runtime.tools import *  # noqa: F401,F403
from garfield_amd.runtime.tools import (  # noqa: F401
    _call_method, _remote_method_async, _remote_method_sync, get_server, get_worker,
)
