"""AdamW (decoupled weight decay, the same "adam" kernel), ref:python_src_quants/optim/adamw.py."""
from .optimizer import Optimizer2State


class AdamW(Optimizer2State):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 optim_bits=32, args=None, min_8bit_size=4096, percentile_clipping=100, block_wise=True,
                 is_paged=False):
        if amsgrad:
            raise NotImplementedError("amsgrad is not supported")
        super().__init__("adam", params, lr, betas, eps, weight_decay, optim_bits, args, min_8bit_size,
                         percentile_clipping, block_wise, is_paged=is_paged)


class AdamW8bit(Optimizer2State):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 optim_bits=32, args=None, min_8bit_size=4096, percentile_clipping=100, block_wise=True,
                 is_paged=False):
        if amsgrad:
            raise NotImplementedError("amsgrad is not supported")
        super().__init__("adam", params, lr, betas, eps, weight_decay, 8, args, min_8bit_size,
                         percentile_clipping, block_wise, is_paged=is_paged)


class AdamW32bit(Optimizer2State):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 optim_bits=32, args=None, min_8bit_size=4096, percentile_clipping=100, block_wise=True,
                 is_paged=False):
        if amsgrad:
            raise NotImplementedError("amsgrad is not supported")
        super().__init__("adam", params, lr, betas, eps, weight_decay, 32, args, min_8bit_size,
                         percentile_clipping, block_wise, is_paged=is_paged)
