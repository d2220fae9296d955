"""Stand-in for ``librosa`` (absent here).  TEST INFRASTRUCTURE: only ``librosa.filters.mel`` is
restated (oracle/_stubs/librosa/filters.py), which Mel-Band-Roformer needs at construction."""
from . import filters  # noqa: F401
