"""Device-resident tables.

``DeviceFrame`` stands where the reference passes a pandas DataFrame of
parameters (``History.get_distribution`` -> ``Transition.fit``,
pyabc/storage/history.py:269-313): the rows live on the GPU as an [n, d]
float64 tensor, columns are the parameter names sorted as pandas' pivot sorts
them.  ``.values`` / ``to_pandas()`` copy to the host on demand only.
"""
import numpy as np
import pandas as pd
import torch


class DeviceFrame:
    def __init__(self, tensor, columns):
        if tensor.dim() == 1:
            tensor = tensor.view(-1, 1)
        self.tensor = tensor
        self.columns = pd.Index(list(columns))

    def __len__(self):
        return self.tensor.shape[0]

    @property
    def shape(self):
        return tuple(self.tensor.shape)

    @property
    def values(self):
        return self.tensor.detach().cpu().numpy()

    def to_pandas(self):
        return pd.DataFrame(self.values, columns=self.columns)

    def __getitem__(self, cols):
        if isinstance(cols, str):
            j = self.columns.get_loc(cols)
            return pd.Series(self.tensor[:, j].cpu().numpy(), name=cols)
        idx = [self.columns.get_loc(c) for c in cols]
        return DeviceFrame(self.tensor[:, idx], cols)

    def __repr__(self):
        return f"<DeviceFrame {self.shape} columns={list(self.columns)}>"


def as_device_matrix(X, columns=None, device=None):
    """(tensor [n, d] f64 on the device, column names) from a DataFrame,
    DeviceFrame, Series, ndarray or tensor.  When ``columns`` is given the
    input's columns are reordered to it (MVN.pdf, multivariatenormal.py:104)."""
    dev = device or torch.device("cuda", torch.cuda.current_device())
    if isinstance(X, DeviceFrame):
        t, cols = X.tensor, list(X.columns)
        if columns is not None and list(columns) != cols:
            t = t[:, [cols.index(c) for c in columns]]
            cols = list(columns)
        return t.to(dev, torch.float64).contiguous(), cols
    if isinstance(X, pd.Series):
        if columns is not None:
            X = X[list(columns)]
        return (torch.as_tensor(np.asarray(X.values, dtype=np.float64),
                                device=dev).view(1, -1), list(X.index))
    if isinstance(X, pd.DataFrame):
        if columns is not None:
            X = X[list(columns)]
        return (torch.as_tensor(np.ascontiguousarray(
            X.values, dtype=np.float64), device=dev), list(X.columns))
    if isinstance(X, torch.Tensor):
        t = X.to(dev, torch.float64)
        if t.dim() == 1:
            t = t.view(1, -1)
        return t.contiguous(), columns
    a = np.atleast_2d(np.asarray(X, dtype=np.float64))
    return torch.as_tensor(np.ascontiguousarray(a), device=dev), columns


def as_device_vector(w, device=None):
    dev = device or torch.device("cuda", torch.cuda.current_device())
    if isinstance(w, torch.Tensor):
        return w.to(dev, torch.float64).contiguous().view(-1)
    return torch.as_tensor(np.ascontiguousarray(np.asarray(w, dtype=np.float64)
                                                ).reshape(-1), device=dev)
