"""Import-compatible entry points for code written against the reference (zenghanfu/dpwa):
``from dpwa.adapters.pytorch import DpwaPyTorchAdapter`` and ``from dpwa.dpwa import
DpwaConnection`` resolve to the MI355X implementation in :mod:`dpwa_amd`, so a training
script switches without editing its imports.  The reference's TCP threads (dpwa/conn.py
RxThread / TxThread) have no counterpart here: on a node the learners pull each other's
snapshots over xGMI, and mixed clusters use ``transport="wire"`` (dpwa_amd/bridge.py)."""
