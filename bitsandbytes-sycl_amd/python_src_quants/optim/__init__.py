"""Optimizers with 8-bit blockwise or fp32 states (ref:python_src_quants/optim/__init__.py)."""
from .adagrad import Adagrad, Adagrad8bit, Adagrad32bit
from .adam import Adam, Adam8bit, Adam32bit
from .adamw import AdamW, AdamW8bit, AdamW32bit
from .lion import Lion, Lion8bit, Lion32bit
from .optimizer import GlobalOptimManager, Optimizer1State, Optimizer2State, Optimizer8bit
from .rmsprop import RMSprop, RMSprop8bit, RMSprop32bit
from .sgd import SGD, SGD8bit, SGD32bit

__all__ = ["Adagrad", "Adagrad8bit", "Adagrad32bit", "Adam", "Adam8bit", "Adam32bit", "AdamW", "AdamW8bit",
           "AdamW32bit", "Lion", "Lion8bit", "Lion32bit", "GlobalOptimManager", "Optimizer1State", "Optimizer2State",
           "Optimizer8bit", "RMSprop", "RMSprop8bit", "RMSprop32bit", "SGD", "SGD8bit", "SGD32bit"]
