from garfield_amd.runtime.byz_worker import ByzWorker  # noqa: F401
