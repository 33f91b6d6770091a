from garfield_amd.runtime.byz_server import ByzServer  # noqa: F401
