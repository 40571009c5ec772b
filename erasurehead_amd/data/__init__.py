"""Data pipeline (L2): reference on-disk formats, synthetic GMM generators, real-dataset preparation."""
from .io import (dataset_dir, load_data, load_sparse_csr, save_matrix, save_sparse_csr, save_vector)
from .source import ArraySource, DataSource, FileSource, SyntheticSource
from .synthetic import DeviceGMM, generate_to_disk
