"""Action preprocessing (reference: components/transforms.py:4-22)."""
import torch


class Transform:
    def transform(self, tensor):
        raise NotImplementedError

    def infer_output_info(self, vshape_in, dtype_in):
        raise NotImplementedError


class OneHot(Transform):
    """One-hot of the last (size-1) dim.  Like the reference, the declared output dtype is
    the INPUT dtype (transforms.py:21-22), so int64 actions give int64 `actions_onehot`."""

    def __init__(self, out_dim):
        self.out_dim = out_dim

    def transform(self, tensor):
        out = torch.zeros(*tensor.shape[:-1], self.out_dim, dtype=torch.float32, device=tensor.device)
        out.scatter_(-1, tensor.long(), 1.0)
        return out

    def infer_output_info(self, vshape_in, dtype_in):
        return (self.out_dim,), dtype_in
