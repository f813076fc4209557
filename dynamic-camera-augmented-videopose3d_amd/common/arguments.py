"""Command-line flags of the FCN evaluation path (reference common/arguments.py:10-105).

The flags the temporal-lifter path reads keep their reference names, short
options and defaults (-d/--dataset, -k/--keypoints, --subjects-test, -a/--actions,
-c/--checkpoint, --evaluate, --by-subject, --use-model, -b/--batch-size,
-s/--stride, --fcn-architecture, --causal, -ch/--channels, --fcn-dropout,
--dense, --disable-optimizations, --downsample).  The other model families'
and the trainer's flags (-e, -lr, -lrd, -r, --checkpoint-frequency, --no-eval) drive the training loop of run.py; the rest are accepted for compatibility and ignored.
Added: --compute-dtype, --trust-checkpoint and the --synthetic-* data options.
"""
import argparse


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="MI355X temporal lifter: evaluation driver")
    a = ap.add_argument
    # data / run selection (reference :13-30)
    a('-d', '--dataset', default='synthetic', type=str, metavar='NAME', help='dataset (synthetic)')
    a('-k', '--keypoints', default='gt', type=str, metavar='NAME', help='2D detections to use')
    a('-str', '--subjects-train', type=str, metavar='LIST')
    a('--subjects-test', type=str, metavar='LIST', help='test subjects, comma separated, or *')
    a('-a', '--actions', default='*', type=str, metavar='LIST', help='actions, comma separated, or *')
    a('-c', '--checkpoint', default='checkpoint', type=str, metavar='PATH', help='checkpoint directory')
    a('--evaluate', default='', type=str, metavar='FILENAME',
      help="checkpoint to evaluate (file name in --checkpoint), or 'synthetic' for seeded weights")
    a('--by-subject', action='store_true', help='break down error by subject')
    a('--use-model', dest='model_name', default='FCN', type=str, help='only FCN runs on this path')
    a('-b', '--batch-size', default=1024, type=int, metavar='N')
    a('-s', '--stride', default=1, type=int, metavar='N')
    a('--downsample', default=1, type=int, metavar='FACTOR')
    # temporal FCN (reference :57-61, :78-79)
    a('--fcn-architecture', dest='fcn_architecture', default='3,3,3,3,3', type=str, metavar='LAYERS')
    a('--causal', action='store_true')
    a('-ch', '--channels', default=1024, type=int, metavar='N')
    a('--fcn-dropout', dest='fcn_dropout', default=0.25, type=float, metavar='P')
    a('--dense', action='store_true')
    a('--disable-optimizations', action='store_true')
    # accepted for compatibility, unused on this path
    for flag, kw in [('--checkpoint-frequency', dict(type=int, default=10)), ('-r', dict(dest='resume', default='')),
                     ('-e', dict(dest='epochs', type=int, default=60)),
                     ('-lr', dict(dest='learning_rate', type=float, default=0.001)),
                     ('-lrd', dict(dest='lr_decay', type=float, default=0.95)),
                     ('--render', dict(action='store_true')), ('--export-training-curves', dict(action='store_true')),
                     ('--no-eval', dict(action='store_true')), ('--subset', dict(type=float, default=1)),
                     ('--viz-subject', dict(type=str)), ('--viz-action', dict(type=str))]:
        a(flag, **kw)
    # added
    a('--compute-dtype', default='fp32', choices=['fp32', 'bf16', 'fp16'],
      help='arithmetic of the conv stack (fp32 = parity path)')
    a('--trust-checkpoint', action='store_true',
      help='allow full unpickling of a checkpoint you created yourself (reference checkpoints '
           'hold a numpy RandomState, which weights_only loading rejects)')
    a('--synthetic-subjects', default=3, type=int)
    a('--synthetic-actions', default=3, type=int)
    a('--synthetic-frames', default=600, type=int)
    a('--joints', default=17, type=int)
    a('--trajectory', action='store_true', help='camera-trajectory conditioned input (J + 6 pairs)')
    a('--seed', default=0, type=int)
    args = ap.parse_args(argv)
    if args.resume and args.evaluate:
        ap.error('--resume and --evaluate cannot be set at the same time')
    return args
