"""Drop-in shim: the reference's `utils` module name -> the HIP GE2E helpers (utils.py:27-132).

``mfccs_and_spec`` (utils.py:138-164, librosa features) is imported by the reference's
``data_load.py:17`` at module load, so the name must exist; the raw-wav featurisation itself is
out of scope and raises only when called.
"""
from pytorch_speaker_verification_amd.utils import calc_loss, get_centroids, get_cossim  # noqa: F401


def mfccs_and_spec(wav_file, wav_process=False, calc_mfccs=False, calc_mag_db=False):
    raise NotImplementedError("mfccs_and_spec (librosa raw-wav features, utils.py:138-164) is out of scope: run the "
                              "reference's data_preprocess.py once and set data.data_preprocessed: true")
