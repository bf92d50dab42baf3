"""Density grids of the visualisation layer:
`kde_1d` / `kde_2d` with the reference's signatures and semantics
(pyabc/visualization/kde.py:19-75, 173-247), evaluated by the device KDE
pass (a3) over the grid points.  Plotting (matplotlib figures, the
`plot_kde_*` wrappers) is out of scope: these return the arrays the
reference's plot functions draw.
"""
import numpy as np
import pandas as pd

from .transition import MultivariateNormalTransition

__all__ = ["kde_1d", "kde_2d", "kde_matrix"]


def _host_frame(df):
    return df if isinstance(df, pd.DataFrame) else pd.DataFrame(df)


def kde_1d(df, w, x, xmin=None, xmax=None, numx=50, kde=None):
    """visualization/kde.py:19-75: fit `kde` (default
    MultivariateNormalTransition(scaling=1)) to df[[x]] with weights w and
    return (x_vals, pdf) on numx points of [xmin, xmax]."""
    df = _host_frame(df)
    if kde is None:
        kde = MultivariateNormalTransition(scaling=1)
    kde.fit(df[[x]], w)
    if xmin is None:
        xmin = df[x].min()
    if xmax is None:
        xmax = df[x].max()
    x_vals = np.linspace(xmin, xmax, num=numx)
    pdf = kde.pdf(pd.DataFrame({x: x_vals}))
    return x_vals, pdf


def kde_2d(df, w, x, y, xmin=None, xmax=None, ymin=None, ymax=None,
           numx=50, numy=50, kde=None):
    """visualization/kde.py:173-247: (X, Y, PDF) on the numy x numx mesh."""
    df = _host_frame(df)
    if kde is None:
        kde = MultivariateNormalTransition(scaling=1)
    kde.fit(df[[x, y]], w)
    if xmin is None:
        xmin = df[x].min()
    if xmax is None:
        xmax = df[x].max()
    if ymin is None:
        ymin = df[y].min()
    if ymax is None:
        ymax = df[y].max()
    X, Y = np.meshgrid(np.linspace(xmin, xmax, num=numx),
                       np.linspace(ymin, ymax, num=numy))
    test = pd.DataFrame({x: X.flatten(), y: Y.flatten()})
    PDF = np.asarray(kde.pdf(test)).reshape(X.shape)
    return X, Y, PDF


def kde_matrix(df, w, limits=None, numx=50, numy=50, kde=None):
    """The grids `plot_kde_matrix` draws (visualization/kde.py:420-489):
    kde_1d on the diagonal, kde_2d for every ordered pair of columns, with
    per-parameter limits (default: the data range).  Returns
    {(x, x): (x_vals, pdf), (x, y): (X, Y, PDF)}."""
    df = _host_frame(df)
    limits = limits or {}
    out = {}
    for x in df.columns:
        lx = limits.get(x, (None, None))
        out[(x, x)] = kde_1d(df, w, x, *lx, numx=numx, kde=kde)
        for y in df.columns:
            if y == x:
                continue
            ly = limits.get(y, (None, None))
            out[(x, y)] = kde_2d(df, w, x, y, lx[0], lx[1], ly[0], ly[1],
                                 numx=numx, numy=numy, kde=kde)
    return out
