"""nicnes: MI355X-native NIC-NES population-evaluation engine (drop-in for the fc_caption NES path
of rubencart/NES-img-captioning). See DESIGN.md and include/nicnes.h."""
from .engine import Engine, pack_ngram, df_table_arrays  # noqa: F401
from ._lib import NicnesError, DecodeFault  # noqa: F401

__all__ = ['Engine', 'pack_ngram', 'df_table_arrays']
