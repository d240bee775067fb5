"""Drop-in shim: the reference's `speech_embedder_net` module name -> the HIP implementation."""
from pytorch_speaker_verification_amd.speech_embedder_net import (  # noqa: F401
    GE2ELoss, SpeechEmbedder, calc_loss, get_centroids, get_cossim)
