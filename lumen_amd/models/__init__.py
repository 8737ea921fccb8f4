"""Model families built on lumen_amd.ops (HIP kernels on GPU, PyTorch reference on CPU)."""
