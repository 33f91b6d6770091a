from garfield_amd.data.datasets import *  # noqa: F401,F403
