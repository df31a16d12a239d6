"""SGD with momentum (kernel "momentum"), ref:python_src_quants/optim/sgd.py."""
from .optimizer import Optimizer1State


def _sgd(cls_bits):
    class _SGD(Optimizer1State):
        def __init__(self, params, lr, momentum=0, dampening=0, weight_decay=0, nesterov=False, optim_bits=32,
                     args=None, min_8bit_size=4096, percentile_clipping=100, block_wise=True):
            if momentum == 0:
                raise NotImplementedError("SGD without momentum is not supported!")
            super().__init__("momentum", params, lr, (momentum, dampening), 0.0, weight_decay,
                             cls_bits or optim_bits, args, min_8bit_size, percentile_clipping, block_wise)
    return _SGD


class SGD(_sgd(None)):
    pass


class SGD8bit(_sgd(8)):
    pass


class SGD32bit(_sgd(32)):
    pass
