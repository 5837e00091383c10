cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_knobs.py 24300 '' '21=256' '21=512' '21=768' '21=1024' '' > gpurun_out/ab9.log 2>&1
