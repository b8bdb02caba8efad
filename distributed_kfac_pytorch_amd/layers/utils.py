"""Plain-PyTorch K-FAC math: the CPU path and the fp32 oracle for HIP kernels.

Every function reproduces the reference's numerics exactly (same op order,
so CPU results are bit-identical to kfac/layers/utils.py of the reference):
  append_bias_ones   ~ kfac/layers/utils.py:4-11
  get_cov            ~ kfac/layers/utils.py:13-43   (C = a^T (a/n), then (C+C^T)/2)
  get_eigendecomp    ~ kfac/layers/utils.py:45-74   (symeig -> linalg.eigh, clip >= 0)
  get_inverse        ~ kfac/layers/utils.py:76-96   (Cholesky inverse of F + damping I)
  get_elementwise_inverse ~ kfac/layers/utils.py:98-105
  reshape_data       ~ kfac/layers/utils.py:107-124
  get_triu/fill_triu ~ kfac/layers/utils.py:126-162
  update_running_avg ~ kfac/layers/utils.py:164-178
The GPU path of the same math lives in ops/ (hand-written HIP kernels).
"""
import torch

__all__ = ['append_bias_ones', 'get_cov', 'get_eigendecomp', 'get_inverse',
           'get_elementwise_inverse', 'reshape_data', 'get_triu', 'fill_triu',
           'update_running_avg', 'extract_patches']


def append_bias_ones(tensor):
    """[..., n] -> [..., n+1] with a trailing column of ones."""
    ones = tensor.new_ones(tensor.shape[:-1] + (1,))
    return torch.cat([tensor, ones], dim=-1)


def get_cov(a, b=None, scale=None):
    """Second moment a^T a / scale (scale defaults to the row count).

    With b given: a^T b / scale (no symmetrisation).
    """
    if a.dim() != 2:
        raise ValueError('Input tensor must have 2 dimensions.')
    if b is not None and a.shape != b.shape:
        raise ValueError('Input tensors must have same shape. Got tensors of '
                         'shape {} and {}.'.format(a.shape, b.shape))
    n = a.size(0) if scale is None else scale
    if b is not None:
        return a.t() @ (b / n)
    c = a.t() @ (a / n)
    return (c + c.t()) / 2.0


def get_eigendecomp(tensor, clip=0.0, concat=True, symmetric=True):
    """Eigendecomposition (ascending eigenvalues, clipped from below by `clip`).

    Returns (Q, d) if concat is False, else [Q | d] of shape (n, n+1).
    """
    if symmetric:
        d, Q = torch.linalg.eigh(tensor)
    else:
        d, Q = torch.linalg.eig(tensor)
        d, Q = d.real, Q.real
    Q = Q.contiguous()  # eigh returns column-major storage; keep broadcasts safe
    if clip is not None:
        d = torch.clamp(d, min=clip)
    if concat:
        return torch.cat([Q, d.unsqueeze(-1)], -1)
    return Q, d


def get_inverse(tensor, damping=None, symmetric=True):
    """(tensor + damping I)^-1 via Cholesky when symmetric."""
    if damping is not None:
        tensor = tensor + torch.diag(tensor.new_full((tensor.shape[0],), damping))
    if symmetric:
        return torch.cholesky_inverse(torch.linalg.cholesky(tensor))
    return torch.inverse(tensor)


def get_elementwise_inverse(vector, damping=None):
    """Reciprocal of the non-zero entries (zeros stay zero)."""
    if damping is not None:
        vector = vector + damping
    out = vector.clone()
    nz = out != 0.0
    out[nz] = torch.reciprocal(out[nz])
    return out


def reshape_data(data_list, batch_first=True, collapse_dims=False):
    """Concatenate hook data along the batch dim; optionally flatten to 2-D."""
    dim = 0 if (batch_first or data_list[0].dim() < 3) else 1
    d = data_list[0] if len(data_list) == 1 else torch.cat(data_list, dim=dim)
    if collapse_dims and d.dim() > 2:
        d = d.reshape(-1, d.shape[-1])
    return d


def get_triu(tensor):
    """Row-major flattened upper triangle (diagonal included)."""
    if tensor.dim() != 2:
        raise ValueError('triu(tensor) requires tensor to be 2 dimensional')
    if tensor.shape[0] > tensor.shape[1]:
        raise ValueError('tensor cannot have more rows than columns')
    r, c = torch.triu_indices(tensor.shape[0], tensor.shape[1], device=tensor.device)
    return tensor[r, c]


def fill_triu(shape, triu_tensor):
    """Inverse of get_triu for a symmetric matrix of `shape`."""
    if len(shape) != 2:
        raise ValueError('shape must be 2 dimensional')
    rows, cols = shape
    out = triu_tensor.new_empty((rows, cols))
    r, c = torch.triu_indices(rows, cols, device=triu_tensor.device)
    out[r, c] = triu_tensor
    out[c, r] = triu_tensor
    return out


def update_running_avg(new, current, alpha=1.0):
    """In place: current = alpha*current + (1-alpha)*new.

    Evaluated as current *= alpha/(1-alpha); current += new; current *= (1-alpha)
    to match the reference bit for bit.
    """
    if alpha != 1:
        current *= alpha / (1 - alpha)
        current += new
        current *= (1 - alpha)


def extract_patches(x, kernel_size, stride, padding):
    """im2col for Conv2d: (B, C, H, W) -> (B, OH, OW, C*kh*kw), columns (c, kh, kw).

    Same layout as the reference's pad/unfold/transpose chain
    (kfac/layers/conv.py:50-70) so conv weight.view(out, -1) lines up.
    """
    if padding[0] + padding[1] > 0:
        x = torch.nn.functional.pad(x, (padding[1], padding[1], padding[0], padding[0]))
    x = x.unfold(2, kernel_size[0], stride[0]).unfold(3, kernel_size[1], stride[1])
    # (B, C, OH, OW, kh, kw) -> (B, OH, OW, C, kh, kw)
    x = x.permute(0, 2, 3, 1, 4, 5).contiguous()
    return x.view(x.size(0), x.size(1), x.size(2), -1)
