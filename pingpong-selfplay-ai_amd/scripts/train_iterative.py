"""scripts/train_iterative.py on the device: generations of a NoisyNet QNet modelB against modelA
and the checkpoint pool, reading config.yaml from the working directory as the reference does.
See pongmi.generations.QNetGenerations for the batching semantics."""
from _common import load_config, parse

if __name__ == "__main__":
    args = parse(__doc__, 512)
    from pongmi.generations import QNetGenerations
    QNetGenerations(load_config(args.config or "config.yaml"), n_arenas=args.arenas, seed=args.seed,
                    check_every=args.check_every, replay_ratio=args.replay_ratio,
                    updates_per_step=args.updates_per_step).run()
