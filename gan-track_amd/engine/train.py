"""YAML entry point of the trainer:  python -m engine.train --config configs/claro_stylegan2-ada.yaml [--set k=v ...]

The reference trains only through click flags (SG3/train_mi_multimodal.py:148-203); its YAML files
(configs/*.yaml) are read by the generation scripts (src/models/gen_images.py:113-119).  This entry reads
the same kind of YAML file and takes the trainer's options from its `trainer_gan:` block, whose keys are
the click flag names (`map-depth` or `map_depth` alike); `--set key=value` overrides one.  The result is
the same `c` as the flags would give (train_mi_multimodal.build_config) -> training_options.json ->
training_loop.  Top-level `seed` is used when the block has none.
"""
import argparse
import sys

import yaml

import train_mi_multimodal as cli


def options_from_yaml(path, overrides=()):
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    block = dict(cfg.get('trainer_gan') or {})
    opts = {k.replace('-', '_'): v for k, v in block.items()}
    if 'seed' not in opts and 'seed' in cfg:
        opts['seed'] = cfg['seed']
    for kv in overrides:
        k, _, v = kv.partition('=')
        opts[k.replace('-', '_')] = yaml.safe_load(v)
    known = set(cli.DEFAULTS) | {'outdir', 'cfg', 'data', 'gpus', 'batch', 'gamma'}
    unknown = sorted(set(opts) - known)
    if unknown:
        raise SystemExit(f'{path}: trainer_gan has keys that are not trainer flags: {unknown}')
    for k in ('aug_opts', 'metrics'):          # YAML lists or the flags' comma strings
        if isinstance(opts.get(k), list):
            opts[k] = ','.join(str(x) for x in opts[k])
    if isinstance(opts.get('modalities'), list):
        opts['modalities'] = ','.join(opts['modalities'])
    return opts


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split('\n')[0])
    ap.add_argument('--config', required=True)
    ap.add_argument('--set', action='append', default=[], metavar='KEY=VALUE')
    ap.add_argument('-n', '--dry-run', action='store_true')
    a = ap.parse_args(argv)
    opts = options_from_yaml(a.config, a.set)
    if a.dry_run:
        opts['dry_run'] = True
    c, desc, outdir, dry_run = cli.build_config(**opts)
    cli.launch_training(c=c, desc=desc, outdir=outdir, dry_run=dry_run)


if __name__ == '__main__':
    sys.exit(main())
