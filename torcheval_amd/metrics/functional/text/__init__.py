"""Text metrics, functional API (parity: functional/text/*.py)."""

from torcheval_amd.metrics.functional.text.helper import (
    _edit_distance,
    _get_errors_and_totals,
    _text_pair_check,
)
from torcheval_amd.metrics.functional.text.word_error_rate import (
    word_error_rate,
    _word_error_rate_update,
    _word_error_rate_compute,
)
from torcheval_amd.metrics.functional.text.word_information_lost import (
    _wil_update,
    _wil_compute,
    word_information_lost,
)
from torcheval_amd.metrics.functional.text.word_information_preserved import (
    word_information_preserved,
    _word_information_preserved_update,
    _word_information_preserved_compute,
)
from torcheval_amd.metrics.functional.text.bleu import (
    bleu_score,
    _bleu_score_update,
    _get_ngrams,
    _bleu_counts_py,
    _bleu_score_compute,
    _calc_brevity_penalty,
)
from torcheval_amd.metrics.functional.text.perplexity import (
    perplexity,
    _perplexity_update,
    _perplexity_compute,
    _perplexity_shape_check,
    _perplexity_label_check,
    _perplexity_input_check,
)

__all__ = [
    "bleu_score",
    "perplexity",
    "word_error_rate",
    "word_information_lost",
    "word_information_preserved",
]
__doc_name__ = "Text Metrics"
