"""Drop-in shim: the reference's `hparam` module name -> pytorch_speaker_verification_amd.hparam."""
from pytorch_speaker_verification_amd.hparam import Dotdict, Hparam, hparam, load_hparam, merge_dict  # noqa: F401
