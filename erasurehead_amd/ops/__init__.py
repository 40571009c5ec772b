"""Device operators (L6): worker gradients, combine+update, evaluation — gfx950 HIP kernels."""
from .eval import auc_columns, loss_sums, predictions
from .grad import DenseGradPlan, SparseGradPlan, choose_cpl
from .precision import PRECISIONS, Precision, get_precision
from .update import combine_update
