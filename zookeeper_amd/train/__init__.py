"""Training: experiments, the step loop, losses, optimizers, metrics and
checkpoint/resume."""

from zookeeper_amd.train.experiment import Experiment, TrainingExperiment
from zookeeper_amd.train.losses import get_loss, softmax_cross_entropy
from zookeeper_amd.train.optimizers import SGD, Adam, FlatOptimizer, OptimizerSpec
from zookeeper_amd.train.trainer import Trainer, prepare_model

__all__ = [
    "Adam",
    "Experiment",
    "FlatOptimizer",
    "get_loss",
    "OptimizerSpec",
    "prepare_model",
    "SGD",
    "softmax_cross_entropy",
    "Trainer",
    "TrainingExperiment",
]
