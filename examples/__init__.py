"""Training examples (reference: examples/ of MLHPC/Distributed_KFAC_Pytorch)."""
