source tools/gpu_steps.sh
export AB_STEPS=20
step parity_nhpa 300 env APN_HIP_LIB=ab/nhpa/libapn_hip.so python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mlp or forward_vs_oracle"
step ab 900 bash tools/ab.sh "APN_AB=cur" "APN_HIP_LIB=ab/nh/libapn_hip.so" "APN_HIP_LIB=ab/nhp/libapn_hip.so" "APN_HIP_LIB=ab/nhpa/libapn_hip.so" "APN_AB=cur2" "APN_HIP_LIB=ab/nhp/libapn_hip.so" "APN_HIP_LIB=ab/nh/libapn_hip.so"
