"""Scheme engine (L4): one master/worker loop for every gradient code + the evaluation epilogue."""
from .evaluate import EvalResult, evaluate
from .trainer import TrainResult, Trainer
