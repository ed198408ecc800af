"""Extract the polygon rings of the reference's own resource `high_risk_zones.geojson`
(src/main/resources, loaded by sncb/tests/LocalTestRunner.java:43 and
sncb/tests/BenchmarkRunner.java:50 for Q1_HighRisk) into a small data fixture, so the GPU
parity test of that caller shape (tests/test_gpu_callers.py) needs no /root/reference at run
time.  Only the coordinates are kept (data, not source).  Run here: python tests/golden/make_callers.py"""
import json
import os

SRC = "/root/reference/src/main/resources/high_risk_zones.geojson"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "high_risk_zones_rings.json")


def main():
    with open(SRC) as f:
        fc = json.load(f)
    polys = []
    for feat in fc["features"]:  # PolygonLoader.loadGeoJsonResourceBuffered: FeatureCollection -> geometries
        g = feat["geometry"]
        assert g["type"] == "Polygon"
        polys.append(g["coordinates"])  # [shell, holes...] as [[x, y], ...]
    with open(OUT, "w") as f:
        json.dump({"source": "src/main/resources/high_risk_zones.geojson", "polygons": polys}, f)
        f.write("\n")
    print(OUT, len(polys))


if __name__ == "__main__":
    main()
