"""Model definitions used by metrics (FID feature extractor) and examples."""

from torcheval_amd.models.inception import FIDInceptionV3, Inception3, inception_v3

__all__ = ["FIDInceptionV3", "Inception3", "inception_v3"]
