"""Command-line flags of run.py (reference common/arguments.py:10-105).

Every reference flag is registered with the reference's spellings (short and long),
dest and default, so a reference command line parses unchanged.  The temporal-FCN
path reads: -d/--dataset, -k/--keypoints, -str/--subjects-train, --subjects-test,
-a/--actions, -c/--checkpoint, --checkpoint-frequency, -r/--resume, --evaluate,
--by-subject, --use-model, -e/--epochs, -b/--batch-size, -lr/--learning-rate,
-lrd/--lr-decay (parsed and unused by the reference's train(), quirk kept in run.py),
-s/--stride, --fcn-architecture, --causal, -ch/--channels, --fcn-dropout, --dense,
--no-eval, --subset, --downsample.  The other model families' flags (LSTM,
Transformer, StackedPoseLifter), tuning and visualisation flags are accepted and
ignored: those paths are outside the temporal-lifter scope.

Differences: -d defaults to 'synthetic' (the reference's 'h36m' default needs
.npz files at a hard-coded path, run.py:48,84; here --data-dir names the directory);
the reference exits on --resume with --evaluate, here argparse reports the error.
Added: --data-dir, --compute-dtype, --trust-checkpoint, --trajectory, --joints,
--seed and the --synthetic-* data options.
"""
import argparse

DATASETS = ("synthetic", "h36m", "CMU", "CMU_3DPW", "3DPW", "humaneva", "custom")


def build_parser():
    ap = argparse.ArgumentParser(description="MI355X temporal lifter: training / evaluation driver")
    a = ap.add_argument
    # General (reference :13-29)
    a('-d', '--dataset', default='synthetic', type=str, metavar='NAME', help='target dataset: ' + ', '.join(DATASETS))
    a('-k', '--keypoints', default='gt', type=str, metavar='NAME', help='2D detections to use')
    a('-str', '--subjects-train', type=str, metavar='LIST', help='training subjects separated by comma')
    a('--subjects-test', type=str, metavar='LIST', help='test subjects separated by comma, or *')
    a('-a', '--actions', default='*', type=str, metavar='LIST', help='actions separated by comma, or *')
    a('-c', '--checkpoint', default='checkpoint', type=str, metavar='PATH', help='checkpoint directory')
    a('--checkpoint-frequency', default=10, type=int, metavar='N', help='create a checkpoint every N epochs')
    a('-r', '--resume', default='', type=str, metavar='FILENAME', help='checkpoint to resume (file name)')
    a('--evaluate', default='', type=str, metavar='FILENAME',
      help="checkpoint to evaluate (file name in --checkpoint), or 'synthetic' for seeded weights")
    a('--render', action='store_true', help='visualize a particular video (not on this path)')
    a('--by-subject', action='store_true', help='break down error by subject (on evaluation)')
    a('--export-training-curves', action='store_true', help='save training curves (not on this path)')
    # Model selection / learning (:32-38)
    a('--use-model', dest='model_name', default='FCN', type=str, help='FCN (TemporalModel), Transformer (CoupledTransformer) or LSTM-Coupled '
      '(CoupledLSTM; --evaluate runs the trajectory lifters over sliding windows)')
    a('-e', '--epochs', default=60, type=int, metavar='N', help='number of training epochs')
    a('-b', '--batch-size', default=1024, type=int, metavar='N', help='batch size in terms of predicted frames')
    a('-lr', '--learning-rate', default=0.001, type=float, metavar='LR', help='initial learning rate')
    a('-lrd', '--lr-decay', default=0.95, type=float, metavar='LR', help='learning rate decay per epoch')
    # LSTM / Transformer / StackedPoseLifter (:40-63): accepted, other model families
    a('--hidden-features', dest='lstm_hidden_features', default=128, type=int, metavar='N')
    a('--lstm-cells', dest='lstm_cells', default=2, type=int, metavar='N')
    a('--lstm-head-architecture', dest='lstm_head_architecture', default='128,128,128', type=str, metavar='X,Y,Z')
    a('--lstm-dropout', dest='lstm_dropout', default=0.25, type=float, metavar='P')
    a('--d-model', dest='d_model', default=128, type=int, metavar='N')
    a('--num-layers', dest='num_layers', default=2, type=int, metavar='N')
    a('--n_heads', dest='n_heads', default=4, type=int, metavar='N')
    a('--dim-feedforward', dest='dim_feedforward', default=128, type=int, metavar='N')
    a('--transformer-head-architecture', dest='transformer_head_architecture', default='128,128,128', type=str,
      metavar='X,Y,Z')
    a('--transformer-dropout', dest='transformer_dropout', default=0.25, type=float, metavar='P')
    a('--stacked-num-layers', dest='stacked_num_layers', default=3, type=int, metavar='N')
    a('--layer-size', dest='layer_size', default=256, type=int, metavar='N')
    a('--stacked-pose-lifter-dropout', dest='stacked_pose_lifter_dropout', default=0.25, type=float, metavar='P')
    a('--transformer-weights', dest='transformer_weights', default='', type=str, metavar='PATH')
    a('--fcn-weights', dest='fcn_weights', default='', type=str, metavar='PATH')
    # Temporal FCN (:55-61)
    a('-s', '--stride', default=1, type=int, metavar='N', help='chunk size to use during training')
    a('--fcn-architecture', dest='fcn_architecture', default='3,3,3,3,3', type=str, metavar='LAYERS',
      help='temporal FCN filter widths separated by comma')
    a('--causal', action='store_true', help='use causal convolutions for real-time processing')
    a('-ch', '--channels', default=1024, type=int, metavar='N', help='number of channels in convolution layers')
    a('--fcn-dropout', dest='fcn_dropout', default=0.25, type=float, metavar='P', help='temporal FCN dropout probability')
    # Experimental (:66-79)
    a('--tune-hyperparameters', action='store_true', help='(not on this path)')
    a('-te', '--tuning-epochs', default=20, type=int, metavar='N')
    a('--subjects-validate', type=str, metavar='LIST')
    a('--subset', default=1, type=float, metavar='FRACTION', help='reduce dataset size by fraction')
    a('--downsample', default=1, type=int, metavar='FACTOR', help='downsample frame rate by factor')
    a('--warmup', default=1, type=int, metavar='N')
    a('--no-eval', action='store_true', help='disable epoch evaluation while training')
    a('--dense', action='store_true', help='use dense convolutions instead of dilated convolutions')
    a('--disable-optimizations', action='store_true', help='disable optimized model for single-frame predictions')
    # Visualization (:82-94): accepted, rendering is not on this path
    a('--viz-subject', type=str, metavar='STR')
    a('--viz-action', type=str, metavar='STR')
    a('--viz-camera', type=int, default=0, metavar='N')
    a('--viz-video', type=str, metavar='PATH')
    a('--viz-skip', type=int, default=0, metavar='N')
    a('--viz-output', type=str, metavar='PATH')
    a('--viz-export', type=str, metavar='PATH')
    a('--viz-bitrate', type=int, default=3000, metavar='N')
    a('--viz-no-ground-truth', action='store_true')
    a('--viz-limit', type=int, default=-1, metavar='N')
    a('--viz-downsample', type=int, default=1, metavar='N')
    a('--viz-size', type=int, default=5, metavar='N')
    # added
    a('--data-dir', default='data', type=str, metavar='PATH',
      help='directory holding data_3d_<dataset>.npz and data_2d_<dataset>_<keypoints>.npz '
           '(the reference hard-codes /vol/bitbucket/bw1222/data/npz)')
    a('--compute-dtype', default='fp32', choices=['fp32', 'f16x3', 'bf16', 'fp16'],
      help='arithmetic of the conv stack (fp32 = parity path; f16x3 = split fp16, fp32-level results on the 16-bit MFMAs)')
    a('--trust-checkpoint', action='store_true',
      help='allow full unpickling of a checkpoint you created yourself (by default only tensors, '
           'plain containers and the numpy RandomState of a run.py checkpoint are admitted)')
    a('--synthetic-subjects', default=3, type=int)
    a('--synthetic-actions', default=3, type=int)
    a('--synthetic-frames', default=600, type=int)
    a('--joints', default=17, type=int, help='joints of the synthetic dataset')
    a('--trajectory', action='store_true', help='camera-trajectory conditioned input (J + 6 pairs)')
    a('--seed', default=0, type=int)
    return ap


def parse_args(argv=None):
    ap = build_parser()
    args = ap.parse_args(argv)
    # reference :97-105
    if args.resume and args.evaluate:
        ap.error('--resume and --evaluate cannot be set at the same time')
    if args.export_training_curves and args.no_eval:
        ap.error('--export-training-curves and --no-eval cannot be set at the same time')
    if args.dataset not in DATASETS:
        ap.error(f'unknown dataset {args.dataset!r} (one of {", ".join(DATASETS)})')
    return args
