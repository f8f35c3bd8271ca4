"""Command line of marlnav_amd, mirroring the reference's
``python -m marlnav`` (marlnav/__main__.py): same arguments and defaults.

Implemented mode: the reward check (``-rc``, utils.py:579-666 via
__main__.py:36-42) on the HIP environment step. Training (MAPPO) and
rendering are the reference's own code and stay there: they take
``marlnav_amd.Env`` as their environment.

    python -m marlnav_amd -rc -se 0            # config-1 reward check
    python -m marlnav_amd -rc -sn 0 -ms 400    # mock scenario 0
"""
import argparse
import sys


def build_parser():
    """The reference's arguments (marlnav/__main__.py:49-132)."""
    p = argparse.ArgumentParser(prog="python -m marlnav_amd",
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    a = p.add_argument
    a('-se', '--seed', type=int, help='value of the random seed (optional, default is None).')
    a('-mx', '--max_x_value', type=float, default=1500.0)
    a('-my', '--max_y_value', type=float, default=750.0)
    a('-fx', '--fig_size_x', type=float, default=10.0)
    a('-fy', '--fig_size_y', type=float, default=5.0)
    a('-pi', '--parallel_index', type=int, default=0)
    a('-ai', '--agent_index', type=int, default=0)
    a('-in', '--interval', type=int, default=10)
    a('-ra', '--random', action='store_true')
    a('-w', '--weights_file', type=str)
    a('-np', '--num_parallel', type=int, default=2)
    a('-na', '--num_agents', type=int, default=3)
    a('-no', '--num_obstacles', type=int, default=3)
    a('-ms', '--max_step', type=int, default=1000)
    a('-el', '--episode_len', type=int, default=200)
    a('-mis', '--min_speed', type=float, default=3.)
    a('-mas', '--max_speed', type=float, default=10.)
    a('-mia', '--min_accel', type=float, default=-0.5)
    a('-maa', '--max_accel', type=float, default=0.5)
    a('-rf', '--risk_factor', type=float, default=0.)
    a('-df', '--distance_factor', type=float, default=0.)
    a('-hf', '--heading_factor', type=float, default=500.)
    a('-tf', '--target_factor', type=float, default=500.)
    a('-sf', '--soft_factor', type=float, default=500.)
    a('-bf', '--bond_factor', type=float, default=10.)
    a('-hs', '--hidden_size', type=int, default=50)
    a('-lr', '--learning_rate', type=float, default=0.001)
    a('-ec', '--ent_const', type=float, default=0.001)
    a('-ep', '--epsilon', type=float, default=0.01)
    a('-g', '--gamma', type=float, default=0.9)
    a('-nt', '--num_total', type=int, default=1000000)
    a('-bl', '--buffer_len', type=int, default=1000)
    a('-ne', '--num_epochs', type=int, default=50)
    a('-bs', '--batch_size', type=int, default=1000)
    a('-re', '--rendering', action='store_true')
    a('-sa', '--sampling_style', type=str, default='sampler')
    a('-rc', '--reward_check', action='store_true')
    a('-sn', '--sampler_num', type=int, default=-1)
    # marlnav_amd only
    a('--rng', choices=('reference', 'native'), default='reference',
      help='re-init randomness: the reference torch RNG stream (bit-compatible '
           'with python -m marlnav) or the in-kernel Philox stream')
    a('--init-noise-device', choices=('auto', 'cpu'), default='auto',
      help="generator of the initializer's agent-noise draw: 'auto' = the env device, as "
           "the reference does on a GPU machine; 'cpu' = as on a CPU-only machine (the "
           "reference's CPU run, BASELINE configs[0])")
    a('--plot-dir', default='plots', help='directory of the saved figures')
    a('--no-plots', action='store_true', help='skip the figures, print the series')
    return p


def main(argv=None):
    import importlib

    import torch
    pkg = importlib.import_module("marl-nav_amd")
    args = build_parser().parse_args(argv)
    if not args.reward_check:
        mode = 'rendering' if args.rendering else 'training'
        print(f"marlnav_amd implements the environment step; {mode} is the reference's "
              "own code (MAPPO / animation): run it with marlnav_amd.Env as its "
              "environment (INTEGRATION.md). Use -rc for the reward check.",
              file=sys.stderr)
        return 2
    if not torch.cuda.is_available():
        print("marlnav_amd needs a HIP device (no CPU fallback)", file=sys.stderr)
        return 1
    device = 'cuda'
    if args.seed is not None:
        pkg.set_all_seeds(args.seed)          # __main__.py:137-138
    env_params = pkg.set_env_params(args, device)
    env_params['rng'] = args.rng
    if args.init_noise_device == 'cpu':
        env_params['init'] = dict(env_params['init'], noise_device='cpu')
    anim = pkg.utils.set_animation_params(args, device)
    env = pkg.Env(env_params)
    series = pkg.utils.check_rews(env, anim['max_step'], anim['parallel_index'],
                                  anim['agent_index'], plot_dir=args.plot_dir,
                                  plot=not args.no_plots)
    if args.no_plots:
        for k, v in series.items():
            print(k, " ".join(f"{x:.9g}" for x in v))
    else:
        print(f"saved figures under {args.plot_dir}/")
    return 0


if __name__ == "__main__":
    sys.exit(main())
