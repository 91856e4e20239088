source tools/gpu_steps.sh
AB_STEPS=20 step ab 900 bash tools/ab.sh "APN_AB=default" "APN_MLP_BLOCKS=8192" "APN_MLP_BLOCKS=12288" "APN_MLP_BLOCKS=24576" "APN_MLP_BLOCKS=32768" "APN_MLP_BLOCKS=3072" "APN_AB=default2"
