"""gale model zoo: network IR, packing, plans and the fp32 reference forward."""

from gale.models.graph import (  # noqa: F401
    AvgPool, Conv, Head, MaxPool, Network, Softmax, build_plan, fold_params, init_params,
    unfolded_params,
    pack_params, param_layout,
)
from gale.models.zoo import MODELS, get_model, lenet5, resnet20, resnet50  # noqa: F401
