"""ArcFace identity encoder on MI355X: the ``netArc`` GHOST loads (arcface_model.iresnet)."""
from .iresnet import IBasicBlock, IResNet, iresnet18, iresnet34, iresnet50, iresnet100  # noqa: F401
from .pipeline import embed_crops, match_faces, normalize_and_torch_batch  # noqa: F401
