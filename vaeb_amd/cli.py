"""Command-line surface of the reference's VAEB.py (/root/reference/VAEB.py:22-38,
471-612), kept key-for-key so vaeb_amd drops in for `python VAEB.py ...`.

Same `command_line_args` / `command_line_flags` dicts (including the misspelt
`full_varational`), the same `--name value` / `--flag` parsing with a warning (not an
error) for unused arguments, the same stdout lines and trace CSV.  Keys ADDED (never
renamed): device, rng, objective, max_eval_rows, trace_dedup, fv_sample, state_file,
resume_file, world_size, dp_scaling, dtype (args) and synthetic (flag).

Data parallelism: `--world_size N` runs N ranks, one process per GPU.
Without a launcher the CLI starts them itself (`python -m vaeb_amd ...` per rank, RANK /
LOCAL_RANK / WORLD_SIZE in the environment, before any GPU call); under torch.distributed.run
the launcher's WORLD_SIZE is used.  Each rank takes its share of every minibatch
(dp_scaling strong: the reference's batch_size split over the ranks, so the steps are the
reference's; weak: batch_size rows per rank), the gradient is all-reduced over RCCL inside
the library, validation is sharded and summed, and only rank 0 prints, traces and saves.
`--dtype` chooses the engine the reference chose with THEANO_FLAGS floatX
(run_on_gpu.sh:2): float32 (default) or bf16.
"""
from __future__ import annotations

import copy
import gzip
import os
import sys
import time

import numpy as np

from . import dp

#   to add another command line argument, add its name as a key and a tuple of its
#   default value and type as the value (VAEB.py:22-36)
command_line_args = {'seed': (15485863, int),
                     'n_latent': (10, int),
                     'n_epochs': (2000, int),
                     'batch_size': (100, int),
                     'L': (1, int),
                     'hidden_unit': (-1, int),
                     'learning_rate': (0.01, float),
                     'trace_file': ('', str),
                     'save_file': ('', str),
                     'load_file': ('', str),
                     'vb_param_file': ('', str),
                     # --- added by vaeb_amd ---
                     'device': (0, int),            # HIP device ordinal
                     'rng': ('philox', str),        # philox (device) | theano (host RandomStreams emulation)
                     'objective': ('sum_prior', str),  # sum_prior (VAEB.py) | mean_map (VAEBfullbayes.py)
                     'max_eval_rows': (10000, int),
                     'trace_dedup': (0, int),       # 1: write each trace row once
                     'fv_sample': (0, int),         # 1 (with --full_varational): weight-posterior sample
                                                    # theta~ = mu + |sigma| zeta (VAEB.py:127-129; extension)
                     'state_file': ('', str),       # native checkpoint (theta + Adagrad + RNG) written at the end
                     'resume_file': ('', str),      # native checkpoint to resume from
                     'world_size': (0, int),        # data-parallel ranks (0: one GPU, no communicator;
                                                    # N >= 1: N ranks with the RCCL all-reduce step)
                     'dp_scaling': ('strong', str), # strong: batch_size split over the ranks; weak: per rank
                     'dtype': ('float32', str)}     # float32 (floatX, run_on_gpu.sh:2) | bf16 | fp16
#   to add a new flag, add its name (VAEB.py:37-38)
command_line_flags = ['continuous', 'generic_estimator', 'full_varational',
                      'synthetic']                 # added: synthetic data when the pickles are absent


def get_arg(arg, args, default, type_):
    """VAEB.py:471-480: consume `--arg value` from the list, else the default."""
    arg = '--' + arg
    if arg in args:
        index = args.index(arg)
        value = args[index + 1]
        del args[index]
        del args[index]
        return type_(value)
    return default


def get_flag(flag, args, prefix='--'):
    """VAEB.py:483-489 (freyFace.py:282-288 spells flags with one dash: prefix '-')."""
    flag = prefix + flag
    have_flag = flag in args
    if have_flag:
        args.remove(flag)
    return have_flag


def parse_args(argv=None, spec=None, flags=None, flag_prefix='--', out=print):
    """VAEB.py:491-504 (spec / flags: another driver's tables, e.g. freyFace.py:20-30, whose
    parse_args (:290-300) does not report unused arguments; out: where the report goes)."""
    args = copy.deepcopy(sys.argv[1:] if argv is None else list(argv))
    arg_dict = {}
    for arg_name, (default, type_) in (spec or command_line_args).items():
        arg_dict[arg_name] = get_arg(arg_name, args, default, type_)
    for flag_name in (flags or command_line_flags):
        arg_dict[flag_name] = get_flag(flag_name, args, flag_prefix)
    if len(args) > 0 and spec is None:
        out('Have unused args: {0}'.format(args))
    return arg_dict


def print_args(args, out=print):
    """VAEB.py:507-512."""
    out('Parameters used:')
    out('--------------------------------------')
    for k, v in args.items():
        out('\t{0}: {1}'.format(k, v))
    out('--------------------------------------')


def load_model(file_name):
    """VAEB.py:514-516 loads a pickled model object; here: a checkpoint's
    (header, params), decoded statically (vaeb_amd.pickle_static)."""
    from .pickle_static import read_mdl
    return read_mdl(file_name)


def save_model(model, file_name):
    """VAEB.py:518-521."""
    model.save(file_name)


def load_dataset(continuous, synthetic=False, splits=2):
    """Data as train_model reads it (VAEB.py:541-556): freyfaces.pkl split 1500 / rest,
    or mnist.pkl.gz's (train, valid) images; both from the working directory.  With
    `synthetic` (or when the file is absent and synthetic is set) the SURVEY 8(d)
    synthetic stand-ins of the same shapes are used."""
    from .pickle_static import read_array_pickle
    from .synthetic import frey_like, mnist_like
    if continuous:
        if os.path.exists('freyfaces.pkl') or not synthetic:
            data = np.asarray(read_array_pickle('freyfaces.pkl'), np.float32)
        else:
            data = frey_like()
        return data[:1500], data[1500:]
    if os.path.exists('mnist.pkl.gz') or not synthetic:
        sets = read_array_pickle('mnist.pkl.gz')
        if splits == 3:   # VAEB.load's form (VAEB.py:237-239)
            return tuple((np.asarray(x, np.float32), np.asarray(y)) for x, y in sets)
        (x_train, _), (x_valid, _), _ = sets
        return np.asarray(x_train, np.float32), np.asarray(x_valid, np.float32)
    x = mnist_like(70000)
    if splits == 3:
        lab = np.zeros(10000, np.int64)
        return (x[:50000], np.zeros(50000, np.int64)), (x[50000:60000], lab), (x[60000:], lab)
    return x[:50000], x[50000:60000]


def _quiet(*a, **k):
    pass


def dp_layout(args):
    """(world, rank, local_rank, communicator wanted) from the args and the launcher's
    environment: world_size 0 with no launcher is one GPU without a communicator (the fused
    step); world_size N >= 1 asks for N ranks with the all-reduce step; a launcher's
    WORLD_SIZE > 1 implies it."""
    world_env, rank, local = dp.env_ranks()
    ws = int(args.get('world_size', 0) or 0)
    if ws < 0:
        raise ValueError('world_size must be >= 0')
    if ws == 0:
        return world_env, rank, local, world_env > 1
    if world_env != ws:
        raise ValueError('--world_size {0} but the launcher started {1} rank(s)'.format(ws, world_env))
    return ws, rank, local, True


def train_model(args):
    """VAEB.py:524-598: build the model, then per epoch shuffle the batch order, run every
    minibatch step (device-side, no per-step host sync), validate, trace and print.  With
    data parallelism every rank runs this loop on its share of each minibatch (the same
    seed, so the same batch order everywhere); rank 0 alone prints, traces and saves."""
    from .model import VAEB
    world, rank, local, use_comm = dp_layout(args)
    say = print if rank == 0 else _quiet
    lead = rank == 0
    np.random.seed(args['seed'])
    n_latent = args['n_latent']
    n_epochs = args['n_epochs']
    continuous = args['continuous']
    batch_size = args['batch_size']
    L = args['L']
    hidden_unit = args['hidden_unit']
    learning_rate = args['learning_rate']
    trace_file = args['trace_file']
    generic_estimator = args['generic_estimator']
    full_varational = args['full_varational']
    save_file = args['save_file']
    vb_param_file = args['vb_param_file']
    kw = dict(device=args.get('device', 0) + local, rng=args.get('rng', 'philox'),
              objective=args.get('objective', 'sum_prior'), max_eval_rows=args.get('max_eval_rows', 10000),
              fv_sample=bool(args.get('fv_sample', 0)), dtype=args.get('dtype', 'float32'))
    B_local = batch_size
    if use_comm:
        B_local, kw['row_offset'], kw['B_global'] = dp.row_split(batch_size, world, rank,
                                                                 args.get('dp_scaling', 'strong'))
        group = dp.init_host_group(world)
        from . import _lib
        kw['comm'] = (dp.comm_uid(group, rank, _lib.Context.comm_unique_id), rank, world)

    say("loading data")
    if hidden_unit < 0:
        hidden_unit = 200 if continuous else 500
    data = load_dataset(continuous, args.get('synthetic', False))
    x_train, x_valid = data

    say("creating the model")
    params = None
    if full_varational:
        from .pickle_static import read_mdl
        _, params = read_mdl(vb_param_file)
    model = VAEB(x_train, continuous, hidden_unit, n_latent, B_local, L, learning_rate, generic_estimator,
                 full_varational, params, **kw)
    if use_comm and model._ctx.comm_count() != world:
        raise RuntimeError('rank {0}: the RCCL communicator holds {1} ranks, expected {2}'.format(
            rank, model._ctx.comm_count(), world))

    if args.get('resume_file'):
        model.load_state(args['resume_file'])
    # x_valid is uploaded once and evaluated on device each epoch (VAEB.py:582)
    model.set_validation_data(x_valid)

    say("learning")
    dedup = bool(args.get('trace_dedup', 0))
    trace = len(trace_file) > 0 and lead
    if trace:
        with open(trace_file, 'w') as f:
            f.write('num_samples,L,Lvalid\n')
    # minibatches of the GLOBAL batch (= batch_size unless dp_scaling weak)
    batch_order = np.arange(int(model.N / getattr(model, 'B_global', model.batch_size)))
    for epoch in range(n_epochs):
        start = time.time()
        np.random.shuffle(batch_order)
        LB = model.update_epoch(batch_order)
        LB /= len(batch_order)
        # VAEB.validate returns the SGVB sum (VAEB.py:418-422), divided here (:582); the
        # mean_map objective's validate already returns the mean (VAEBfullbayes.py:161-165)
        LBvalidation = model.validate_resident()
        if model.objective != "mean_map":
            LBvalidation /= x_valid.shape[0]
        if trace:
            with open(trace_file, 'a') as f:
                f.write('{0},{1},{2}\n'.format(model.N * (epoch + 1), LB, LBvalidation))
        say("Epoch %s : [Lower bound: %s, time: %s]" % (epoch, LB, time.time() - start))
        say("          [Lower bound on validation set: %s]" % LBvalidation)
        if trace and not dedup:  # the reference writes every row twice (VAEB.py:591-593)
            with open(trace_file, 'a') as f:
                f.write('{0},{1},{2}\n'.format(model.N * (epoch + 1), LB, LBvalidation))
    if len(save_file) > 0 and lead:
        model.save(save_file)
    if args.get('state_file'):
        # a collective with the sharded DP optimizer (the Adagrad shards are gathered): every
        # rank joins, rank 0 writes (rank 0 alone blocked in the all-gather)
        model.save_state(args['state_file'] if lead else None)
    if use_comm and group is not None:
        # every rank leaves together: the others wait here while rank 0 writes the .mdl and the
        # trace, so the launcher's straggler deadline (dp.spawn_ranks) only ever measures a rank
        # that is really stuck, never rank 0's lead-only tail
        group.barrier()
    return model, data


def main(argv=None):
    """VAEB.py:601-608.  `--world_size N` (N > 1) without a launcher: start the N rank
    processes first (no GPU call in this one) and return their exit code."""
    argv = sys.argv[1:] if argv is None else list(argv)
    ws = get_arg('world_size', list(argv), 0, int)
    if ws > 1 and 'WORLD_SIZE' not in os.environ:
        rc = dp.spawn_ranks(ws, dp.module_cmd(argv),
                            env_extra={'PYTHONPATH': os.pathsep.join(
                                [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))] +
                                ([os.environ['PYTHONPATH']] if os.environ.get('PYTHONPATH') else []))})
        if rc:
            raise SystemExit(rc)
        return None, None
    say = print if dp.env_ranks()[1] == 0 else _quiet
    args = parse_args(argv, out=say)
    print_args(args, out=say)
    if len(args['load_file']) == 0:
        model, data = train_model(args)
    else:
        from .model import VAEB
        model, data = VAEB.load(args['load_file'])
    return model, data


if __name__ == '__main__':
    main()
