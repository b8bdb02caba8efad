"""K-FAC-friendly modules (reference: kfac/modules/__init__.py)."""
from .lstm import LSTMCellBase, LSTMCellKFAC, LSTMCell, LSTMLayer, LSTM

__all__ = ['LSTMCellBase', 'LSTMCellKFAC', 'LSTMCell', 'LSTMLayer', 'LSTM']
