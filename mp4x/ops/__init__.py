"""Native kernel bindings (HIP / CDNA4) and their torch-facing wrappers."""
from . import native  # noqa: F401
