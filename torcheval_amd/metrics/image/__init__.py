"""Image metrics, class API (parity: metrics/image/{psnr,fid}.py).

``FrechetInceptionDistance`` is imported lazily (``torcheval_amd.metrics.FrechetInceptionDistance``
resolves on first access), so importing the metrics package never needs a vision library.
"""

from torcheval_amd.metrics.image.psnr import PeakSignalNoiseRatio

__all__ = ["FrechetInceptionDistance", "PeakSignalNoiseRatio"]
__doc_name__ = "Image Metrics"


def __getattr__(name):
    if name == "FrechetInceptionDistance":
        from torcheval_amd.metrics.image.fid import FrechetInceptionDistance

        return FrechetInceptionDistance
    raise AttributeError(name)
