"""Result table of ``dedispersion_search``.

The reference returns ``astropy.table.Table({'DM','max','std','snr','rebin'})``
(``dedispersion.py:248``).  astropy is used when importable; otherwise this minimal
column table with the same column names, order and dtypes is returned
(``table['snr']``, ``table.colnames``, ``len(table)``, ``table[i]`` row access).
"""
import numpy as np


class Table:
    def __init__(self, cols):
        self._cols = {k: np.asarray(v) for k, v in cols.items()}
        lens = {len(v) for v in self._cols.values()}
        if len(lens) > 1:
            raise ValueError("columns of unequal length")

    @property
    def colnames(self):
        return list(self._cols)

    def __len__(self):
        return len(next(iter(self._cols.values()))) if self._cols else 0

    def __getitem__(self, key):
        if isinstance(key, str):
            return self._cols[key]
        return {k: v[key] for k, v in self._cols.items()}

    def __contains__(self, key):
        return key in self._cols

    def keys(self):
        return self._cols.keys()

    def __repr__(self):
        return f"<Table rows={len(self)} cols={self.colnames}>"


def make_table(cols):
    try:
        from astropy.table import Table as AstropyTable
    except Exception:  # astropy absent (this image): dict-like fallback
        return Table(cols)
    return AstropyTable(cols)
