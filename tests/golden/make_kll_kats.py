"""Writes tests/golden/kll_kats.json: the reference's KLLSketch known answers
(T/KLL/KLLProfileTest.scala:47-157; fixtures FixtureSupport.scala:137-147 and :162-196). Each case is
the non-NULL column values in row order, the KLL parameters and the expected BucketDistribution
(buckets, parameters, compactor data). Run: python tests/golden/make_kll_kats.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = [
    {"name": "NumericFractionalValues", "source": "T/KLL/KLLProfileTest.scala:49-80", "type": "double",
     "values": [1.0, 2.0, 3.0, 4.0, 5.0, 6.0], "nulls": 0, "params": [2, 0.64, 2],
     "buckets": [[1.0, 3.5, 4], [3.5, 6.0, 2]], "parameters": [0.64, 2.0], "data": [[5.0, 6.0], [1.0, 3.0]],
     "profile": {"completeness": 1.0, "approxNumDistinct": 6, "mean": 3.5, "maximum": 6.0, "minimum": 1.0,
                 "sum": 21.0, "stdDev": 1.707825127659933}},
    {"name": "NumericFractionalValuesForKLL", "source": "T/KLL/KLLProfileTest.scala:82-116", "type": "double",
     "values": [float(i) for i in range(1, 31)], "nulls": 0, "params": [2, 0.64, 2],
     "buckets": [[1.0, 15.5, 16], [15.5, 30.0, 14]], "parameters": [0.64, 2.0],
     "data": [[27.0, 28.0, 29.0, 30.0], [25.0], [1.0, 6.0, 10.0, 15.0, 19.0, 23.0]],
     "profile": {"completeness": 1.0, "approxNumDistinct": 30, "mean": 15.5, "maximum": 30.0, "minimum": 1.0,
                 "sum": 465.0, "stdDev": 8.65544144839919}},
    {"name": "ShortTypeWithNull", "source": "T/KLL/KLLProfileTest.scala:118-155", "type": "short",
     "values": [1, 2, 3, 4, 5, 6], "nulls": 1, "params": [2, 0.64, 2],
     "buckets": [[1.0, 3.5, 4], [3.5, 6.0, 2]], "parameters": [0.64, 2.0], "data": [[5.0, 6.0], [1.0, 3.0]]},
]

if __name__ == "__main__":
    with open(os.path.join(HERE, "kll_kats.json"), "w") as f:
        json.dump(CASES, f, indent=1)
