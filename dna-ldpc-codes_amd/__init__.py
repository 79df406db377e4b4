"""MI355X-native batched LDPC decoder (drop-in for the ldpc.exe step of
sjpark0905/DNA-LDPC-codes).  See ldpc_amd.py and include/ldpc_amd.h.

The directory name contains hyphens, so import it by path::

    import importlib.util, sys
    spec = importlib.util.spec_from_file_location(
        "dna_ldpc_codes_amd", "dna-ldpc-codes_amd/__init__.py",
        submodule_search_locations=["dna-ldpc-codes_amd"])
    pkg = importlib.util.module_from_spec(spec); sys.modules[spec.name] = pkg
    spec.loader.exec_module(pkg)

or simply put dna-ldpc-codes_amd/ on sys.path and ``import ldpc_amd``.
"""
from . import ldpc_amd  # noqa: F401
from . import synth  # noqa: F401
from .ldpc_amd import Graph, Engine, decode, decode_files, graph, device_count  # noqa: F401
