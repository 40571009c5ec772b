"""Model families (L6 math spec): L2 logistic regression and least squares."""
from .losses import (LEAST_SQUARES, LOGISTIC, LOSS_NAMES, UpdateRule, least_squares_grad, logistic_grad,
                     logistic_loss, mse, roc_auc, worker_grad)
