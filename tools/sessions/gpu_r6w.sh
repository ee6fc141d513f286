# round 6: knockout timing of the latent step's end chains (lab only: the dW1 / dW2 TN launch
# and / or the fold backward skipped) to see which chain binds the step
set -o pipefail
bash tools/ab_variants.sh r6w latent latent_train.hip 3
