#!/bin/bash
# BASELINE config 5 rehearsal on one GPU: lr x wd grid of the ImageNet-shape
# E18 task, 4 concurrent @task runs packed onto the box's GPU (--runs-per-gpu 4).
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
export ZK_SWEEP_DIR=gpurun_out/r1az_sweep
gpu_step 600 gpurun_out/r1az_sweep.log python examples/train_imagenet.py TrainImageNet \
  --grid 'learning_rate=[1e-3,2e-3]' --grid 'optimizer.weight_decay=[0.0,1e-5]' --runs-per-gpu 4 \
  batch_size=128 steps_per_epoch=40 validation_steps=4 log_every=10 device_pool=4 \
  "output_dir='/tmp/r1az_runs'" print_summary=False
echo done >> gpurun_out/progress.txt
du -sh /tmp/r1az_runs/TrainImageNet/* >> gpurun_out/progress.txt 2>&1 || true
