"""MI355X drop-in for the reference ``network`` package (AEI_Net, AADLayer, AAD_ResBlk)."""
from .AADLayer import AAD_ResBlk, AADLayer, AddBlocksSequential  # noqa: F401
from .AEI_Net import AADGenerator, AEI_Net, MLAttrEncoder, conv4x4, deconv4x4, weight_init  # noqa: F401
