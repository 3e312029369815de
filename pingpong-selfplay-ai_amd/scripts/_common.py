"""Shared entry-point plumbing for the training scripts: import paths, config, CLI."""
import argparse
import os
import sys

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if PKG not in sys.path:
    sys.path.insert(0, PKG)


def parse(description, default_arenas):
    ap = argparse.ArgumentParser(description=description)
    ap.add_argument("--arenas", type=int, default=default_arenas, help="arenas stepped in lockstep on the device")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--check-every", type=int, default=4, help="vector steps between episode-budget checks")
    ap.add_argument("--config", default=None, help="config file (default: the reference's name, in the CWD)")
    ap.add_argument("--replay-ratio", type=float, default=1.0,
                    help="updates per pushed transition (1.0 = the reference's one update per env step)")
    ap.add_argument("--updates-per-step", type=int, default=None,
                    help="updates per vector step (overrides --replay-ratio)")
    return ap.parse_args()


def load_config(path):
    import yaml
    with open(path, "r") as f:
        return yaml.safe_load(f)
