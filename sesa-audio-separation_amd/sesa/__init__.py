"""sesa -- MI355X-native chunked source-separation engine (drop-in for the
test4373/SESA-Audio-Separation separation hot path).  See DESIGN.md at the repo root."""
__version__ = "0.1.0"

from .config import ConfigDict, load_config, prefer_target_instrument  # noqa: F401
