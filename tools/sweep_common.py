"""Shared check of the sweep tools (tools/sweep.py, slot_sweep.py, tx_sweep.py; not part of the
product). The product library accepts only the default values of the sweep-only tunables
unroll, packets, nontemporal and frames (aipstack_chksum_tune returns EINVAL otherwise): their
variants are compiled only into a build made with

    tools/build_variant.sh NAME -DAIPSTACK_ALL_VARIANTS      (-> tools/build/lib_NAME.so)

and passed to the tool with --lib tools/build/lib_NAME.so."""
import sys

SWEEP_ONLY_DEFAULTS = {"unroll": (0,), "packets": (0,), "nontemporal": (1,), "frames": (0, 4)}


def all_variants(lib) -> bool:
    """Whether the loaded library was built with -DAIPSTACK_ALL_VARIANTS."""
    ok = lib.aipstack_chksum_tune(b"unroll", 1) == 0
    lib.aipstack_chksum_tune(b"unroll", 0)
    return ok


def require_variants(lib, variants) -> None:
    """Exit with the build recipe when a variant sets a sweep-only tunable to a value the
    loaded library rejects. `variants`: iterable of {tunable: value} dicts."""
    need = sorted({k for v in variants for k, x in v.items()
                   if k in SWEEP_ONLY_DEFAULTS and x not in SWEEP_ONLY_DEFAULTS[k]})
    if need and not all_variants(lib):
        sys.exit(f"these variants set {', '.join(need)}: the product library accepts only their "
                 "defaults. Build tools/build_variant.sh NAME -DAIPSTACK_ALL_VARIANTS and pass "
                 "--lib tools/build/lib_NAME.so")
