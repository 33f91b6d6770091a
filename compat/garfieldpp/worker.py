from garfield_amd.runtime.worker import Worker  # noqa: F401
