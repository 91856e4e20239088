source tools/gpu_steps.sh
export AB_STEPS=10
step ab 900 bash tools/ab.sh "APN_AB=cur" "APN_HIP_LIB=ab/l1w/libapn_hip.so" "APN_HIP_LIB=ab/nop/libapn_hip.so" "APN_HIP_LIB=ab/norec/libapn_hip.so"
