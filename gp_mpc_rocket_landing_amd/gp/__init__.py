"""GP surfaces (reference src/gp): kernels, exact / sparse GPs, features, structured GPs."""
from .exact_gp import ExactGP, GPPrediction, MultiOutputExactGP
from .features import (AtmosphereModel, CombinedFeatureExtractor, RocketFeatureExtractor,
                       RotationalFeatureExtractor, Simple3DoFFeatureExtractor,
                       TranslationalFeatureExtractor)
from .kernels import (RBF, SE_ARD, Matern32, Matern52, ProductKernel, SquaredExponential,
                      SquaredExponentialARD, SumKernel, WhiteNoise, create_matern_kernel)
from .online_update import (DataBuffer, DataPoint, OnlineGPUpdater, OnlineStructuredGPUpdater,
                            OnlineUpdateConfig, ResidualCollector)
from .sparse_gp import MultiOutputSparseGP, SparseGP
from .structured_gp import Simple3DoFGP, StructuredGPConfig, StructuredRocketGP

__all__ = ["ExactGP", "GPPrediction", "MultiOutputExactGP", "AtmosphereModel", "CombinedFeatureExtractor",
           "RocketFeatureExtractor", "RotationalFeatureExtractor", "Simple3DoFFeatureExtractor",
           "TranslationalFeatureExtractor", "RBF", "SE_ARD", "Matern32", "Matern52", "ProductKernel",
           "SquaredExponential", "SquaredExponentialARD", "SumKernel", "WhiteNoise", "create_matern_kernel",
           "MultiOutputSparseGP", "SparseGP", "Simple3DoFGP", "StructuredGPConfig",
           "StructuredRocketGP", "DataBuffer", "DataPoint", "OnlineGPUpdater",
           "OnlineStructuredGPUpdater", "OnlineUpdateConfig", "ResidualCollector"]
