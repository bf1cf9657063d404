"""MI355X-native autoencoder collaborative filtering (I-AutoRec / omnidirectional denoising AE).

Drop-in for the hot path of Epist/omnidirectional_collaborative_filtering: the
``data_reader`` batch API (data_reader.py) and the ``omni_model`` / Keras-Model training surface
(model.py, train.py), implemented on hand-written HIP kernels for gfx950 behind a C ABI
(include/ocf.h, libocf.so).  PyTorch-ROCm provides device memory, streams and torch.distributed.
"""
from . import _lib, metrics, optimizers  # noqa: F401
from .optimizers import SGD, Adagrad, Adam, RMSprop  # noqa: F401

# Module layout mirrors the reference: ``from omnidirectional_collaborative_filtering_amd.data_reader import
# data_reader`` and ``from omnidirectional_collaborative_filtering_amd.model import omni_model``.
__all__ = ["omni_model", "Model", "Adagrad", "RMSprop", "Adam", "SGD", "metrics"]


def __getattr__(name):
    # torch-dependent modules load lazily so the package imports (and the C ABI can be checked)
    # without pulling torch in
    if name in ("omni_model", "Model", "EarlyStopping"):
        from . import model
        return getattr(model, name)
    raise AttributeError(name)
