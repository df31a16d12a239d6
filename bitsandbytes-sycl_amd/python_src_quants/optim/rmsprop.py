"""RMSprop (kernel "rmsprop", betas = (alpha, momentum)), ref:python_src_quants/optim/rmsprop.py."""
from .optimizer import Optimizer1State


def _rmsprop(cls_bits):
    class _RMSprop(Optimizer1State):
        def __init__(self, params, lr=1e-2, alpha=0.99, eps=1e-8, weight_decay=0, momentum=0, centered=False,
                     optim_bits=32, args=None, min_8bit_size=4096, percentile_clipping=100, block_wise=True):
            if alpha == 0:
                raise NotImplementedError("RMSprop with alpha==0.0 is not supported!")
            if centered:
                raise NotImplementedError("Centered RMSprop is not supported!")
            super().__init__("rmsprop", params, lr, (alpha, momentum), eps, weight_decay, cls_bits or optim_bits,
                             args, min_8bit_size, percentile_clipping, block_wise)
    return _RMSprop


class RMSprop(_rmsprop(None)):
    pass


class RMSprop8bit(_rmsprop(8)):
    pass


class RMSprop32bit(_rmsprop(32)):
    pass
