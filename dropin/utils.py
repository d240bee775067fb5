"""Drop-in shim: the reference's `utils` GE2E helpers -> the HIP implementation."""
from pytorch_speaker_verification_amd.utils import calc_loss, get_centroids, get_cossim  # noqa: F401
