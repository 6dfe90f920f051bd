"""final_reward of the reference's own runs, per cell and seed (data, transcribed from
/root/reference/artifacts/combined_validated_data-final-run.csv: lr 3e-4, clip 0.2, entropy 0.005,
8 epochs; batch_size 64 and 32; the PE conditions at d_embed 4).  The reference's plain
"shuffled" condition observes sorted rows (make_env's setdefault quirk), so its rows
equal the sorted ones and are not listed separately.  CSV rows: sorted h256 bs64 :230-232, bs32
:221-223; shuffled_rope h256 d4 bs64 :176-178."""

REFERENCE = {
    ("sorted", 256): {"bs64": {42: 136.8270, 1042: 127.8022, 2042: 132.6172},
                      "bs32": {42: 122.0790, 1042: 120.0389, 2042: 123.3965}},
    ("sorted", 384): {"bs64": {42: 135.6114, 1042: 113.3057, 2042: 108.0399},
                      "bs32": {42: 86.7809, 1042: 96.9049, 2042: 130.7995}},
    ("sorted", 512): {"bs64": {42: 118.0541, 1042: 110.4705, 2042: 127.7685},
                      "bs32": {42: 105.2060, 1042: 115.7746, 2042: 112.0424}},
    ("shuffled_rope", 256): {"bs64": {42: 136.0069, 1042: 82.4615, 2042: 125.5533},
                             "bs32": {42: 91.2034, 1042: 120.1456, 2042: 97.2532}},
    ("shuffled_distpe", 256): {"bs64": {42: 136.0069, 1042: 82.4615, 2042: 125.5533},
                               "bs32": {42: 91.2034, 1042: 120.1456, 2042: 97.2532}},
    ("shuffled_rankpe", 256): {"bs64": {42: 83.2977, 1042: 119.7457, 2042: 119.0862},
                               "bs32": {42: 116.2577, 1042: 76.9021, 2042: 140.8664}},
}
