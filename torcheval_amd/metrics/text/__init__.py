"""Text class metrics (parity: metrics/text/*.py)."""

from torcheval_amd.metrics.text._sum_states import _SumStates
from torcheval_amd.metrics.text.bleu import BLEUScore
from torcheval_amd.metrics.text.perplexity import Perplexity
from torcheval_amd.metrics.text.word_error_rate import WordErrorRate
from torcheval_amd.metrics.text.word_information_lost import WordInformationLost
from torcheval_amd.metrics.text.word_information_preserved import WordInformationPreserved

__all__ = [
    "BLEUScore",
    "Perplexity",
    "WordErrorRate",
    "WordInformationLost",
    "WordInformationPreserved",
]
__doc_name__ = "Text Metrics"
