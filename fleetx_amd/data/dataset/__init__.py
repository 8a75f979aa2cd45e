"""Dataset registry."""
from .gpt_dataset import (GPTDataset, SyntheticGPTDataset, LM_Eval_Dataset,  # noqa: F401
                          Lambada_Eval_Dataset)
from .ernie_dataset import ErnieDataset  # noqa: F401

DATASETS = {
    "GPTDataset": GPTDataset,
    "ErnieDataset": ErnieDataset,
    "SyntheticGPTDataset": SyntheticGPTDataset,
    "LM_Eval_Dataset": LM_Eval_Dataset,
    "Lambada_Eval_Dataset": Lambada_Eval_Dataset,
}


def register_dataset(name, cls):
    DATASETS[name] = cls
    return cls


def _register_optional():
    from .vision_dataset import GeneralClsDataset, ImageFolder, CIFAR, SyntheticImageDataset
    from .multimodal_dataset import ImagenDataset, SyntheticImagenDataset
    for c in (GeneralClsDataset, ImageFolder, CIFAR, SyntheticImageDataset, ImagenDataset,
              SyntheticImagenDataset):
        DATASETS[c.__name__] = c


_register_optional()
