"""Drop-in shim: the reference's `data_load` module name (data_load.py:19-85) -> this package's loader."""
from pytorch_speaker_verification_amd.data_load import SpeakerDatasetTIMIT, SpeakerDatasetTIMITPreprocessed  # noqa: F401
