/*
 * HipKnnWindowFunction -- the window body that replaces PointPointKNNQuery.windowBased's keyed
 * per-cell apply + windowAll merge (PointPointKNNQuery.java:159-200, KNNQuery.java:213-272)
 * with one device evaluation per window.  NOT COMPILED here (no JDK in the build image); see
 * INTEGRATION.md for the binding and tests/test_shim_native.py for the C core it calls.
 *
 * The reference:
 *   filteredPoints.keyBy(gridID).window(SlidingProcessingTimeWindows.of(size, slide))
 *       .apply(per-cell bounded PQ)                              // :159-192
 *       .windowAll(SlidingProcessingTimeWindows.of(size, slide))
 *       .apply(new kNNWinAllEvaluationPointStream(k));          // :198-200
 * becomes
 *   pointStream.windowAll(SlidingProcessingTimeWindows.of(size, slide))
 *       .apply(new HipKnnWindowFunction(grid, queryPoint, r, k));
 * The cell filter (:143-149) is part of the device evaluation, so the stream is not filtered
 * first.  The output is the reference's Tuple3(window start, window end, PQ of (Point,
 * distance)) with the same PQ order (Comparators.inTuplePointDistanceComparator: largest
 * distance at the head) and the same Point instances the window held.
 *
 * gridArgs are the UniformGrid(int n, minX, maxX, minY, maxY) constructor's arguments
 * {n, minX, maxX, minY, maxY} (UniformGrid.java:74-85): that constructor keeps the bounds as
 * given and sets cellLength = (maxX - minX) / n, which gf_grid_make restates.
 */
package GeoFlink.native_;

import GeoFlink.spatialObjects.Point;
import GeoFlink.utils.Comparators;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.configuration.Configuration;
import org.apache.flink.streaming.api.functions.windowing.RichAllWindowFunction;
import org.apache.flink.streaming.api.windowing.windows.TimeWindow;
import org.apache.flink.util.Collector;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.PriorityQueue;

public class HipKnnWindowFunction
    extends RichAllWindowFunction<Point, Tuple3<Long, Long, PriorityQueue<Tuple2<Point, Double>>>, TimeWindow> {

  private final double[] gridArgs;
  private final double qx, qy, radius;
  private final int k;
  private final int device;

  private transient long ctx, plan;
  private transient ByteBuffer bx, by, bo;
  private transient long[] outObjID, outIdx;
  private transient double[] outDist;
  private transient ArrayList<Point> points;
  private transient String[] objIDs;

  public HipKnnWindowFunction(double[] gridArgs, Point queryPoint, double radius, int k, int device) {
    this.gridArgs = gridArgs.clone();
    this.qx = queryPoint.point.getX();
    this.qy = queryPoint.point.getY();
    this.radius = radius;
    this.k = k;
    this.device = device;
  }

  @Override
  public void open(Configuration parameters) {
    ctx = GeoFlinkHip.ctxCreate(device);
    plan = GeoFlinkHip.knnPlan(ctx, gridArgs, qx, qy, radius, k);
    outObjID = new long[k];
    outIdx = new long[k];
    outDist = new double[k];
    points = new ArrayList<>();
    grow(1 << 16);
  }

  @Override
  public void close() {
    if (bo != null) GeoFlinkHip.pinnedFree(bo);
    bo = null;
    if (plan != 0) GeoFlinkHip.knnPlanDestroy(plan);
    if (ctx != 0) GeoFlinkHip.ctxDestroy(ctx);
    plan = ctx = 0;
  }

  private void grow(int n) {
    bx = ByteBuffer.allocateDirect(8 * n).order(ByteOrder.nativeOrder());
    by = ByteBuffer.allocateDirect(8 * n).order(ByteOrder.nativeOrder());
    // the objID keys in pinned memory: the kernels read only the candidates' keys through the
    // mapping, so a window crosses PCIe at 16 B per point (x, y) instead of 24
    if (bo != null) GeoFlinkHip.pinnedFree(bo);
    bo = GeoFlinkHip.pinnedBuffer(8L * n).order(ByteOrder.nativeOrder());
    objIDs = new String[n];
  }

  @Override
  public void apply(TimeWindow window, Iterable<Point> input,
                    Collector<Tuple3<Long, Long, PriorityQueue<Tuple2<Point, Double>>>> out) {
    points.clear();
    for (Point p : input) points.add(p);
    final int n = points.size();
    if (bx.capacity() < 8 * n) grow(n + n / 4);
    for (int i = 0; i < n; i++) {
      Point p = points.get(i);
      bx.putDouble(8 * i, p.point.getX());
      by.putDouble(8 * i, p.point.getY());
      objIDs[i] = p.objID;
    }
    // Point.objID Strings -> keys (the kNN merge dedupes by String.equals, KNNQuery.java:232-251)
    long[] keys = GeoFlinkHip.intern(ctx, objIDs, n);
    bo.asLongBuffer().put(keys, 0, n);

    int m = GeoFlinkHip.knnWindow(ctx, plan, bx, by, bo, n, outObjID, outDist, outIdx, k);

    PriorityQueue<Tuple2<Point, Double>> pq =
        new PriorityQueue<Tuple2<Point, Double>>(k, new Comparators.inTuplePointDistanceComparator());
    for (int j = 0; j < m; j++) pq.offer(new Tuple2<Point, Double>(points.get((int) outIdx[j]), outDist[j]));
    out.collect(Tuple3.of(window.getStart(), window.getEnd(), pq));
  }
}
