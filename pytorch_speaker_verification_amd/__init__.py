"""MI355X-native (gfx950) GE2E speaker-embedding training path.

Drop-in for the hot path of hwidong-na/PyTorch_Speaker_Verification
(SpeechEmbedder + GE2ELoss + the training step); see DESIGN.md and INTEGRATION.md.
The compute runs in libsv_ge2e.so (hand-written HIP, C ABI in include/sv_ge2e.h).
"""
from .hparam import hparam  # noqa: F401
from .speech_embedder_net import GE2ELoss, SpeechEmbedder, calc_loss, get_centroids, get_cossim  # noqa: F401
from ._lib import PersistentRecurrenceError  # noqa: F401
from .ops import check_persistent_status  # noqa: F401
from .trainer import GE2ETrainer  # noqa: F401

__all__ = ["hparam", "SpeechEmbedder", "GE2ELoss", "get_centroids", "get_cossim", "calc_loss", "GE2ETrainer",
           "PersistentRecurrenceError", "check_persistent_status"]
