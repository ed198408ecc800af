/*
 * HipRangeWindowFunction -- the window body that replaces the keyed range apply of
 * PointPointRangeQuery.windowBased (PointPointRangeQuery.java:119-187) and
 * PointPolygonRangeQuery.windowBased (PointPolygonRangeQuery.java:138-205) with one device
 * evaluation per window.  NOT COMPILED here (no JDK in the build image); see INTEGRATION.md and
 * tests/test_shim_native.py (test_java_call_sequences drives this class's native sequence through
 * the C core on the GPU and checks it against the oracle).
 *
 * The reference:
 *   pointStream.filter(cell in C u G)                                    // :135-140
 *       .keyBy(gridID).window(SlidingProcessingTimeWindows.of(size, slide))
 *       .apply(guaranteed cell -> collect; candidate cell -> distance <= r)  // :144-187
 * becomes
 *   pointStream.windowAll(SlidingProcessingTimeWindows.of(size, slide))
 *       .apply(new HipRangeWindowFunction(gridArgs, queryPoints, r, approximate, device));
 * The cell filter, the keyBy and the per-cell apply are the device evaluation (rangePlan once:
 * the G / C cell sets of :119-125; rangeWindow per window).  The callers in the reference are range
 * queries: StreamingJob.java:260,270 and sncb/mobility/MN_Q1.java:63 (point queries),
 * sncb/queries/Q1_HighRisk.java:74 (polygon queries, HipRangeWindowFunction.forPolygons).
 *
 * Output: the window's emitted Points (the instances the window held), in window order; the
 * reference's per-cell keyed apply emits them in a Flink-dependent order.  Approximate point
 * queries with |Q| > 1 emit a candidate-cell point once per query point, as the reference's loop
 * does (PointPointRangeQuery.java:158-161; rangeWindowMulti).
 */
package GeoFlink.native_;

import GeoFlink.spatialObjects.Point;
import GeoFlink.spatialObjects.Polygon;
import org.apache.flink.configuration.Configuration;
import org.apache.flink.streaming.api.functions.windowing.RichAllWindowFunction;
import org.apache.flink.streaming.api.windowing.windows.TimeWindow;
import org.apache.flink.util.Collector;

import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.Set;

public class HipRangeWindowFunction extends RichAllWindowFunction<Point, Point, TimeWindow> {

  private final double[] gridArgs;
  private final double radius;
  private final boolean approximate;
  private final int device;
  private final double[] qx, qy;     // point queries
  private final HipColumns.Csr poly; // polygon queries

  private transient long ctx, plan;
  private transient HipColumns cols;
  private transient ByteBuffer out, multi;
  private transient ArrayList<Point> points;

  /** PointPointRangeQuery.run(pointStream, Set<Point> queryPointSet, r) */
  public HipRangeWindowFunction(double[] gridArgs, Set<Point> queryPoints, double radius, boolean approximate,
                                int device) {
    this.gridArgs = gridArgs.clone();
    this.radius = radius;
    this.approximate = approximate;
    this.device = device;
    this.qx = new double[queryPoints.size()];
    this.qy = new double[queryPoints.size()];
    int i = 0;
    for (Point q : queryPoints) {
      qx[i] = q.point.getX();
      qy[i++] = q.point.getY();
    }
    this.poly = null;
  }

  private HipRangeWindowFunction(double[] gridArgs, Set<Polygon> polygons, double radius, boolean approximate,
                                 int device, boolean unused) {
    this.gridArgs = gridArgs.clone();
    this.radius = radius;
    this.approximate = approximate;
    this.device = device;
    this.qx = this.qy = null;
    this.poly = new HipColumns.Csr(polygons);
  }

  /** PointPolygonRangeQuery.run(pointStream, Set<Polygon> queryPolygonSet, r) */
  public static HipRangeWindowFunction forPolygons(double[] gridArgs, Set<Polygon> polygons, double radius,
                                                   boolean approximate, int device) {
    return new HipRangeWindowFunction(gridArgs, polygons, radius, approximate, device, true);
  }

  @Override
  public void open(Configuration parameters) {
    ctx = GeoFlinkHip.ctxCreate(device);
    plan = poly == null
        ? GeoFlinkHip.rangePlan(ctx, gridArgs, qx, qy, radius, approximate)
        : GeoFlinkHip.rangePolygonPlan(ctx, gridArgs, poly.ringOff, poly.vertOff, poly.vx, poly.vy, radius,
                                       approximate);
    cols = new HipColumns(false);
    points = new ArrayList<>();
  }

  @Override
  public void close() {
    if (plan != 0) GeoFlinkHip.rangePlanDestroy(plan);
    if (ctx != 0) GeoFlinkHip.ctxDestroy(ctx);
    plan = ctx = 0;
  }

  @Override
  public void apply(TimeWindow window, Iterable<Point> input, Collector<Point> neighbors) {
    final int n = HipColumns.list(input, points).size();
    cols.fill(ctx, points);
    out = HipColumns.ints(out, Math.max(1, n / 8));
    long count = GeoFlinkHip.rangeWindow(ctx, plan, cols.x, cols.y, n, out, out.capacity() / 4);
    if (count > out.capacity() / 4) {  // more emitted points than the buffer: once more, large enough
      out = HipColumns.ints(null, count);
      count = GeoFlinkHip.rangeWindow(ctx, plan, cols.x, cols.y, n, out, out.capacity() / 4);
    }
    long nm = 0;
    if (approximate && qx != null && qx.length > 1) {
      multi = HipColumns.ints(multi, Math.max(1, count));
      nm = GeoFlinkHip.rangeWindowMulti(ctx, plan, multi, multi.capacity() / 4);
    }
    // the emitted points ascending; a multiplicity point (also ascending, a subset) |Q| times
    int j = 0;
    for (int i = 0; i < count; i++) {
      final int p = out.getInt(4 * i);
      final Point pt = points.get(p);
      neighbors.collect(pt);
      if (j < nm && multi.getInt(4 * j) == p) {
        for (int r = 1; r < qx.length; r++) neighbors.collect(pt);
        j++;
      }
    }
  }
}
