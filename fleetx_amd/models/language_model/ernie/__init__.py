from .model import (ErnieModel, ErnieForPretraining, ErniePretrainingCriterion,  # noqa: F401
                    ErnieForMaskedLM, ErnieForMultipleChoice, mlm_mask)
