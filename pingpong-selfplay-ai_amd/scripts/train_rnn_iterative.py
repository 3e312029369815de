"""scripts/train_rnn_iterative.py on the device: generations of a QNetRNN modelB (DRQN) with resume
from the latest-state checkpoint, reading config_rnn.yaml from the working directory as the
reference does. See pongmi.generations.RNNGenerations for the batching semantics."""
from _common import load_config, parse

if __name__ == "__main__":
    args = parse(__doc__, 64)
    from pongmi.generations import RNNGenerations
    RNNGenerations(load_config(args.config or "config_rnn.yaml"), n_arenas=args.arenas, seed=args.seed,
                   check_every=args.check_every, replay_ratio=args.replay_ratio,
                   updates_per_step=args.updates_per_step).run()
