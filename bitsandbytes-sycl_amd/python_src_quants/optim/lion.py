"""Lion (kernel "lion"), ref:python_src_quants/optim/lion.py."""
from .optimizer import Optimizer1State


def _lion(cls_bits):
    class _Lion(Optimizer1State):
        def __init__(self, params, lr=1e-4, betas=(0.9, 0.99), weight_decay=0, optim_bits=32, args=None,
                     min_8bit_size=4096, percentile_clipping=100, block_wise=True, is_paged=False):
            super().__init__("lion", params, lr, betas, 0.0, weight_decay, cls_bits or optim_bits, args,
                             min_8bit_size, percentile_clipping, block_wise, is_paged=is_paged)
    return _Lion


class Lion(_lion(None)):
    pass


class Lion8bit(_lion(8)):
    pass


class Lion32bit(_lion(32)):
    pass
