"""Model tools (parity: torcheval/tools/__init__.py)."""

from torcheval_amd.tools.flops import FlopTensorDispatchMode
from torcheval_amd.tools.module_summary import (
    get_module_summary,
    get_summary_table,
    ModuleSummary,
    prune_module_summary,
)

__all__ = [
    "FlopTensorDispatchMode",
    "get_module_summary",
    "get_summary_table",
    "ModuleSummary",
    "prune_module_summary",
]
__doc_name__ = "Tools"
