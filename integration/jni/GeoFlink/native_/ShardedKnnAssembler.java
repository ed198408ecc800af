/*
 * ShardedKnnAssembler -- joins the nranks ShardedKnnParts of one window (keyed by window end) into
 * the reference's output record Tuple3(window start, window end, PriorityQueue<Tuple2<Point,
 * Double>>) under Comparators.inTuplePointDistanceComparator, as PointPointKNNQuery.windowBased
 * emits it (PointPointKNNQuery.java:195-200, KNNQuery.java:213-272).  The selection already
 * happened on the GPUs: every part carries the merged ranks of its band's entries, so this only
 * places m entries.  NOT COMPILED here (no JDK in the build image).
 */
package GeoFlink.native_;

import GeoFlink.spatialObjects.Point;
import GeoFlink.utils.Comparators;
import org.apache.flink.api.common.state.ListState;
import org.apache.flink.api.common.state.ListStateDescriptor;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.configuration.Configuration;
import org.apache.flink.streaming.api.functions.KeyedProcessFunction;
import org.apache.flink.util.Collector;

import java.util.ArrayList;
import java.util.PriorityQueue;

public class ShardedKnnAssembler
    extends KeyedProcessFunction<Long, ShardedKnnPartial, Tuple3<Long, Long, PriorityQueue<Tuple2<Point, Double>>>> {

  private final int k;
  private transient ListState<ShardedKnnPartial> parts;

  public ShardedKnnAssembler(int k) { this.k = k; }

  @Override
  public void open(Configuration parameters) {
    parts = getRuntimeContext().getListState(new ListStateDescriptor<>("gf-knn-parts", ShardedKnnPartial.class));
  }

  @Override
  public void processElement(ShardedKnnPartial part, Context c,
                             Collector<Tuple3<Long, Long, PriorityQueue<Tuple2<Point, Double>>>> out) throws Exception {
    parts.add(part);
    final ArrayList<ShardedKnnPartial> have = new ArrayList<>();
    for (ShardedKnnPartial p : parts.get()) have.add(p);
    if (have.size() < part.nranks) return;  // wait for every rank's part of this window
    parts.clear();
    final PriorityQueue<Tuple2<Point, Double>> pq =
        new PriorityQueue<Tuple2<Point, Double>>(k, new Comparators.inTuplePointDistanceComparator());
    for (ShardedKnnPartial p : have)
      for (int j = 0; j < p.points.size(); j++) pq.offer(new Tuple2<Point, Double>(p.points.get(j), p.dist.get(j)));
    out.collect(Tuple3.of(part.windowStart, part.windowEnd, pq));
  }
}
