/*
 * HipPolygonJoinFunction -- the window body that replaces PointPolygonJoinQuery.windowBased
 * (PointPolygonJoinQuery.java:154-213): the polygon stream replicated to each polygon's own
 * guaranteed and candidate cells (JoinQuery.getReplicatedPolygonQueryStream, JoinQuery.java:
 * 93-115), the cell-keyed window join and the point-polygon distance filter, as one device join
 * per window (polygonJoinWindow = gf_join_ppoly).  NOT COMPILED here (no JDK in the build image);
 * see INTEGRATION.md and tests/test_shim_native.py (test_java_call_sequences).
 *
 *   points.coGroup(polygons).where(p -> 0).equalTo(q -> 0)
 *       .window(SlidingProcessingTimeWindows.of(size, slide))
 *       .apply(new HipPolygonJoinFunction(gridArgs, r, approximate, device));
 * The point and polygon grids must be the same grid (gf_join_ppoly).  Output: Tuple2(point,
 * polygon) of the window's own instances.
 */
package GeoFlink.native_;

import GeoFlink.spatialObjects.Point;
import GeoFlink.spatialObjects.Polygon;
import org.apache.flink.api.common.functions.RichCoGroupFunction;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.configuration.Configuration;
import org.apache.flink.util.Collector;

import java.util.ArrayList;

public class HipPolygonJoinFunction extends RichCoGroupFunction<Point, Polygon, Tuple2<Point, Polygon>> {

  private final double[] gridArgs;
  private final double radius;
  private final boolean approximate;
  private final int device;

  private transient long ctx;
  private transient HipColumns cols;
  private transient ArrayList<Point> points;
  private transient ArrayList<Polygon> polygons;

  public HipPolygonJoinFunction(double[] gridArgs, double radius, boolean approximate, int device) {
    this.gridArgs = gridArgs.clone();
    this.radius = radius;
    this.approximate = approximate;
    this.device = device;
  }

  @Override
  public void open(Configuration parameters) {
    ctx = GeoFlinkHip.ctxCreate(device);
    cols = new HipColumns(false);
    points = new ArrayList<>();
    polygons = new ArrayList<>();
  }

  @Override
  public void close() {
    if (ctx != 0) GeoFlinkHip.ctxDestroy(ctx);
    ctx = 0;
  }

  @Override
  public void coGroup(Iterable<Point> pointIn, Iterable<Polygon> polygonIn, Collector<Tuple2<Point, Polygon>> out) {
    final int n = HipColumns.list(pointIn, points).size();
    if (n == 0 || HipColumns.list(polygonIn, polygons).isEmpty()) return;
    cols.fill(ctx, points);
    final HipColumns.Csr csr = new HipColumns.Csr(polygons);  // this window's polygon side
    final long[] pairs = GeoFlinkHip.polygonJoinWindow(ctx, gridArgs, cols.x, cols.y, n, csr.ringOff, csr.vertOff,
                                                       csr.vx, csr.vy, radius, approximate);
    for (int i = 0; i < pairs.length; i += 2)
      out.collect(Tuple2.of(points.get((int) pairs[i]), polygons.get((int) pairs[i + 1])));
  }
}
