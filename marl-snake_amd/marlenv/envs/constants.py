RGB_CHANNEL = 3       # reference envs/constants.py:1
FEATURE_CHANNEL = 8   # reference envs/constants.py:2
