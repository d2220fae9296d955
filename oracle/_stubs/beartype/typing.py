"""``beartype.typing`` re-exports ``typing`` (stand-in; TEST INFRASTRUCTURE)."""
from typing import *  # noqa: F401,F403
