"""recommender_system_amd — MI355X-native CTR forward path.

Drop-in for the embedding-lookup + feature-interaction forward path of
Hcyand/recommender_system (FM second order, PNN inner product, DCN CrossNet,
DIN attention), as hand-written gfx950 HIP kernels behind a C-ABI
(include/rs_capi.h, librs_hip.so) with a Python host layer that keeps the
reference's Keras layer / model names and signatures.
"""
from . import _lib  # noqa: F401
from .layers import (AFMLayer, Attention, AttentionLayer, BatchNormalization, CrossLayer, Dense, Dice,  # noqa: F401
                     DNNLayer, EmbedLayer, FFMLayer, FMLayer, InnerProductLayer, InteractionLayer,
                     OuterProductLayer, sigmoid_combine)
from .models import AFM, DCN, DIN, FFM, FM, NFM, PNN, DeepFM  # noqa: F401
from .dataset import create_criteo_dataset, denseFeature, features_dict, sparseFeature  # noqa: F401

__version__ = "0.1.0"
