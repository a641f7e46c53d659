from torcheval_amd.utils.device import copy_data_to_device
from torcheval_amd.utils.random_data import (
    get_rand_data_binary,
    get_rand_data_binned_binary,
    get_rand_data_multiclass,
    get_rand_data_multilabel,
)

__all__ = [
    "copy_data_to_device",
    "get_rand_data_binary",
    "get_rand_data_binned_binary",
    "get_rand_data_multiclass",
    "get_rand_data_multilabel",
]
