"""GPT under the auto-parallel front end.

Parity: reference ``gpt/auto/auto_module.py:30-80``, ``auto_utils.py:24-150``
and ``auto_model.py:30-659`` (C22, C32): the module builds a ``Mesh`` from
``Distributed`` (dims ``[pp, dp, mp]``), fills ``ffn_hidden_size`` and the
data ``num_samples``, builds the GPT network and annotates it like the
reference — QKV / FFN1 weights ``[None, mp]``, out-proj / FFN2 weights
``[mp, None]``, word embedding ``[mp, None]`` — then checks the annotations
against the materialised tensor-parallel layers.  ``GPTPretrainingCriterionAuto``
is the vocab-parallel masked-mean cross entropy.

With ``Engine.auto_mode: full`` the degrees are not taken from the YAML but
chosen by :func:`fleetx_amd.parallel.auto.planner.plan` for the world size
(``tools/auto.py`` applies the plan before the process groups are built).
"""
import copy

from .....parallel import topology as topo
from .....parallel.auto.mesh import Mesh, shard_tensor, verify_annotations
from .....parallel.auto.partition import lower
from .....utils.log import logger
from ...language_module import GPTModule
from ...utils import process_data_configs
from ..model import GPTForPretraining, GPTPretrainingCriterion


class GPTPretrainingCriterionAuto(GPTPretrainingCriterion):
    def __init__(self, mesh=None, cfg=None):
        super().__init__(cfg)
        self.mesh = mesh


def annotate_gpt(model, mesh):
    """Reference shard specs (``auto_model.py``) on the built GPT network:
    QKV / FFN1 ``[None, mp]``, out-proj / FFN2 ``[mp, None]``, word embedding
    ``[mp, None]``, and every decoder layer placed on its pipeline sub-mesh
    ``mesh[stage]`` (``auto_model.py:601-610``)."""
    pm = mesh.process_mesh
    mp = mesh.mp
    n = 0
    num_layers = None
    for name, mod in model.named_modules():
        w = getattr(mod, "weight", None)
        if w is None or w.dim() != 2:
            continue
        if name.endswith(("qkv_proj", "fc1")):
            shard_tensor(w, pm, [None, mp])
        elif name.endswith(("out_proj", "fc2")):
            shard_tensor(w, pm, [mp, None])
        elif name.endswith("word_embeddings"):
            shard_tensor(w, pm, [mp, None])
        else:
            continue
        n += 1
    layers = getattr(getattr(model, "gpt", None), "layers", None)
    if layers is not None:
        num_layers = len(layers)
        stages = mesh.stages(num_layers)
        for i, layer in enumerate(layers):
            layer._fx_stage = stages[i]
            layer._fx_mesh = mesh[stages[i]]
    return n


class GPTModuleAuto(GPTModule):
    def process_configs(self, configs):
        configs = super().process_configs(configs)
        d = configs.Distributed
        self.mesh = Mesh(dict(pp_degree=d.pp_degree, dp_degree=d.dp_degree * d.sharding.sharding_degree,
                              mp_degree=d.mp_degree))
        if configs.Model.get("ffn_hidden_size") is None:
            configs.Model["ffn_hidden_size"] = 4 * configs.Model.hidden_size
        process_data_configs(configs)
        return configs

    def _serial_model(self):
        """The annotated serial network (whole weights, one-rank mp world)."""
        cfg = copy.deepcopy(self.gpt_config)
        cfg.sequence_parallel = False
        with topo.serial_scope():
            serial = GPTForPretraining(cfg)
        annotate_gpt(serial, self.mesh)
        return serial

    def get_model(self):
        model = super().get_model()
        q = self.configs.get("Quantization")
        if q is not None and q.get("enable", False):
            # QAT wraps the layers: keep the runtime's own partitioning, check it
            n = annotate_gpt(model, self.mesh)
            checked = verify_annotations(model)
            logger.info("auto-parallel mesh %s: %d annotated weights (%d verified, QAT)"
                        % (self.mesh.process_mesh, n, checked))
            return model
        # semi-auto lowering: the annotations of the serial network decide how
        # every tensor is split (parallel/auto/partition.py)
        serial = self._serial_model()
        layout = lower(serial, model, self.mesh)
        self.auto_layout = layout
        logger.info("auto-parallel mesh %s: lowered %d tensors from the annotated serial network "
                    "(tensor parallel over %s x%d, %d layers stage-annotated)"
                    % (self.mesh.process_mesh, layout["lowered"], layout["tp_dim"],
                       layout["tp_degree"], len(layout["stages"])))
        del serial
        return model

    def get_loss_fn(self):
        return GPTPretrainingCriterionAuto(self.mesh, self.gpt_config)

    @property
    def hcg(self):
        return topo.get_hcg()


def apply_plan(configs, world):
    """``auto_mode: full`` -> fill the Distributed / batch / recompute knobs from the planner."""
    from .....parallel.auto.planner import plan_from_config, describe
    p = plan_from_config(configs, world)
    d = configs.Distributed
    d["dp_degree"], d["mp_degree"], d["pp_degree"] = p.dp, p.mp, p.pp
    d.sharding["sharding_degree"] = p.sharding
    d.sharding["sharding_stage"] = max(1, p.sharding_stage)
    configs.Global["micro_batch_size"] = p.micro_batch
    configs.Model["use_recompute"] = p.recompute
    configs.Engine["use_recompute"] = p.recompute
    logger.info(describe(p))
    return copy.deepcopy(p)
