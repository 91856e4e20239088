source tools/gpu_steps.sh
AB_STEPS=20 step ab 600 bash tools/ab.sh "APN_AB=base" "APN_HIP_LIB=ab/b9occ8/libapn_hip.so" "APN_AB=base2" "APN_HIP_LIB=ab/b9occ8/libapn_hip.so"
