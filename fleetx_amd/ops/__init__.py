"""Hot-path ops: HIP/CDNA4 kernels on GPU tensors, reference math on CPU."""
from .norm import add_layer_norm, layer_norm, layer_norm_keep_input, FusedLayerNorm, col_sum  # noqa: F401
from .elementwise import bias_gelu, bias_dropout_add, dropout  # noqa: F401
from .attention import (flash_attention, flash_attention_qkvpacked, attention_reference,  # noqa: F401
                        decode_attention)
from .loss_embed import softmax_cross_entropy, embedding  # noqa: F401
from .quant import fake_quant  # noqa: F401
from .sampling import fused_sample  # noqa: F401
from .softmax import (fused_softmax, softmax_mask_fuse,  # noqa: F401
                      softmax_mask_fuse_upper_triangle)
from . import _lib  # noqa: F401
from .groupnorm import group_norm_silu, GroupNormSiLU  # noqa: F401,E402
