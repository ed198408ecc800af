/*
 * HipSlidingKnnFunction -- sliding kNN through the device pane engine (gf_knn_sliding_*):
 * the reference's SlidingProcessingTimeWindows.of(size, slide) kNN (PointPointKNNQuery.java:
 * 158,198-200) re-evaluates every point size/slide times; here Flink cuts the stream into
 * tumbling panes of gcd(size, slide) and each pane is evaluated ONCE on the device, a window's
 * result being the top-k-distinct merge of its panes' records (identical to evaluating the window
 * whole).  NOT COMPILED here (no JDK in the build image); tests/test_shim_native.py
 * (test_sliding_knn) drives the same C calls on C5's shape and checks every window.
 *
 *   pointStream.windowAll(TumblingProcessingTimeWindows.of(Time.milliseconds(paneMs)))
 *       .process(new HipSlidingKnnFunction(gridArgs, queryPoint, r, k, sizeMs, slideMs, 0));
 *
 * paneMs = gcd(sizeMs, slideMs) (also GeoFlinkHip.knnSlidingPaneMs).  Output: the reference's
 * Tuple3(window start, window end, PQ of (Point, distance)), emitted when the pane that closes
 * the window arrives (panes Flink does not fire -- no points -- are pushed empty when the next
 * pane arrives).
 */
package GeoFlink.native_;

import GeoFlink.spatialObjects.Point;
import GeoFlink.utils.Comparators;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.configuration.Configuration;
import org.apache.flink.streaming.api.functions.windowing.ProcessAllWindowFunction;
import org.apache.flink.streaming.api.windowing.windows.TimeWindow;
import org.apache.flink.util.Collector;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayDeque;
import java.util.ArrayList;
import java.util.PriorityQueue;

public class HipSlidingKnnFunction
    extends ProcessAllWindowFunction<Point, Tuple3<Long, Long, PriorityQueue<Tuple2<Point, Double>>>, TimeWindow> {

  private final double[] gridArgs;
  private final double qx, qy, radius;
  private final int k;
  private final long sizeMs, slideMs;
  private final int device;

  private transient long ctx, plan, sliding, paneMs, lastPane, pushed;
  private transient int panesPerWindow;
  /* the Points of the latest panes, with their first position in the pushed stream */
  private transient ArrayDeque<Object[]> panes;
  private transient ByteBuffer bx, by, bo;
  private transient long[] outObjID, outIdx;
  private transient double[] outDist;

  public HipSlidingKnnFunction(double[] gridArgs, Point queryPoint, double radius, int k, long sizeMs, long slideMs,
                               int device) {
    this.gridArgs = gridArgs.clone();
    this.qx = queryPoint.point.getX();
    this.qy = queryPoint.point.getY();
    this.radius = radius;
    this.k = k;
    this.sizeMs = sizeMs;
    this.slideMs = slideMs;
    this.device = device;
  }

  @Override
  public void open(Configuration parameters) {
    ctx = GeoFlinkHip.ctxCreate(device);
    plan = GeoFlinkHip.knnPlan(ctx, gridArgs, qx, qy, radius, k);
    sliding = GeoFlinkHip.knnSlidingCreate(ctx, plan, sizeMs, slideMs);
    paneMs = GeoFlinkHip.knnSlidingPaneMs(sliding);
    panesPerWindow = (int) (sizeMs / paneMs);
    lastPane = Long.MIN_VALUE;
    pushed = 0;
    panes = new ArrayDeque<>();
    outObjID = new long[k];
    outIdx = new long[k];
    outDist = new double[k];
    grow(1 << 16);
  }

  @Override
  public void close() {
    if (sliding != 0) GeoFlinkHip.knnSlidingDestroy(sliding);
    if (plan != 0) GeoFlinkHip.knnPlanDestroy(plan);
    if (ctx != 0) GeoFlinkHip.ctxDestroy(ctx);
    sliding = plan = ctx = 0;
  }

  private void grow(int n) {
    bx = ByteBuffer.allocateDirect(8 * n).order(ByteOrder.nativeOrder());
    by = ByteBuffer.allocateDirect(8 * n).order(ByteOrder.nativeOrder());
    bo = ByteBuffer.allocateDirect(8 * n).order(ByteOrder.nativeOrder());
  }

  @Override
  public void process(Context context, Iterable<Point> elements,
                      Collector<Tuple3<Long, Long, PriorityQueue<Tuple2<Point, Double>>>> out) {
    final long pane = context.window().getStart() / paneMs;
    if (lastPane != Long.MIN_VALUE)
      for (long p = lastPane + 1; p < pane; p++) push(p, new ArrayList<Point>(), out);  // panes without points
    ArrayList<Point> pts = new ArrayList<>();
    for (Point p : elements) pts.add(p);
    push(pane, pts, out);
    lastPane = pane;
  }

  private void push(long pane, ArrayList<Point> pts, Collector<Tuple3<Long, Long, PriorityQueue<Tuple2<Point, Double>>>> out) {
    final int n = pts.size();
    if (bx.capacity() < 8 * n) grow(n + n / 4);
    String[] objIDs = new String[n];
    for (int i = 0; i < n; i++) {
      Point p = pts.get(i);
      bx.putDouble(8 * i, p.point.getX());
      by.putDouble(8 * i, p.point.getY());
      objIDs[i] = p.objID;
    }
    if (n > 0) bo.asLongBuffer().put(GeoFlinkHip.intern(ctx, objIDs, n), 0, n);
    panes.addLast(new Object[] {pushed, pts});
    pushed += n;
    while (panes.size() > panesPerWindow) panes.removeFirst();

    final long end = GeoFlinkHip.knnSlidingPush(ctx, sliding, pane, bx, by, bo, n);
    if (end < 0) return;
    int m = GeoFlinkHip.knnSlidingDecode(ctx, sliding, end, outObjID, outDist, outIdx, k);
    PriorityQueue<Tuple2<Point, Double>> pq =
        new PriorityQueue<Tuple2<Point, Double>>(k, new Comparators.inTuplePointDistanceComparator());
    for (int j = 0; j < m; j++) pq.offer(new Tuple2<Point, Double>(pointAt(outIdx[j]), outDist[j]));
    out.collect(Tuple3.of(end - sizeMs, end, pq));
  }

  /* idx = position in the pushed stream -> the Point (it lies in one of the window's panes) */
  @SuppressWarnings("unchecked")
  private Point pointAt(long idx) {
    for (Object[] e : panes) {
      long base = (Long) e[0];
      ArrayList<Point> pts = (ArrayList<Point>) e[1];
      if (idx >= base && idx < base + pts.size()) return pts.get((int) (idx - base));
    }
    throw new IllegalStateException("kNN result outside the window's panes: " + idx);
  }
}
