"""Identity of the search kernel's code, so that measured artefacts (the PMC traffic summary
under profiles/) are only reported for the kernel they were measured on."""
import hashlib
from pathlib import Path

CSRC = Path(__file__).resolve().parent / "csrc"
SEARCH_KERNEL_SOURCES = ("hastar_kernels.hip", "hastar_device.h", "hastar_layout.h", "rbtree_dev.h", "glibc_mathf.h",
                         "hastar_kernels.h", "Makefile")


def search_kernel_hash() -> str:
    """sha256 (first 16 hex digits) over the sources hastar_search_kernel is compiled from."""
    h = hashlib.sha256()
    for name in SEARCH_KERNEL_SOURCES:
        h.update(name.encode())
        h.update((CSRC / name).read_bytes())
    return h.hexdigest()[:16]
