source tools/gpu_steps.sh
export AB_STEPS=20
step ab 900 bash tools/ab.sh "APN_KNN_MASK=1" "APN_KNN_MASK=1 APN_KNN_PTS=2" "APN_KNN_MASK=0" "APN_KNN_MASK=0 APN_KNN_PTS=2" "APN_KNN_MASK=1"
