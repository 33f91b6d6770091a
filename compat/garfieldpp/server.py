from garfield_amd.runtime.server import Server  # noqa: F401
