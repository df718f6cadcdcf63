# Round 6 (last part): retrain the sink run that crossed peak / RMS 100 (lr 2e-3, wd 0.2, BOS
# windows; 14.5 min instead of 16 so that training and the pipeline pass fit one call - the checkpoint cannot leave the
# box) and run BASELINE configs 3-5 through the pipeline on it, incl. config 5's MSE-allocated head-group plans.
OUT=${OUT:-r06g} TRAIN_MIN=14.5 TRAIN_TO=930 LR=2e-3 WD=0.2 SKIP_SWEEP=1 WINDOWS=768 bash scripts/gpu_r06d_sink.sh
