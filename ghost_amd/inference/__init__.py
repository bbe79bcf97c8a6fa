"""Drop-ins for the swap-batch boundary of utils/inference (faceshifter_run.py, core.py)."""
from .core import swap_identity_frames, transform_target_to_torch  # noqa: F401
from .faceshifter_run import faceshifter_batch, faceshifter_batch_u8  # noqa: F401
from .graphed import GraphedSwap  # noqa: F401
