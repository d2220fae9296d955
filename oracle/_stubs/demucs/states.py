"""demucs.states restated (see package docstring): only ``capture_init``."""
import functools


def capture_init(init):
    """Record the constructor arguments on the instance (used for checkpoint serialization)."""

    @functools.wraps(init)
    def __init__(self, *args, **kwargs):
        self._init_args_kwargs = (args, kwargs)
        init(self, *args, **kwargs)

    return __init__
