source tools/gpu_steps.sh
step ab 600 bash tools/ab_c5.sh "APN_AB=cur" "APN_LBS_BLOCKS_PER_CU=8" "APN_HIP_LIB=ab/w5/libapn_hip.so APN_LBS_BLOCKS_PER_CU=5" "APN_HIP_LIB=ab/w6/libapn_hip.so APN_LBS_BLOCKS_PER_CU=6" "APN_HIP_LIB=ab/w6/libapn_hip.so APN_LBS_BLOCKS_PER_CU=12"
