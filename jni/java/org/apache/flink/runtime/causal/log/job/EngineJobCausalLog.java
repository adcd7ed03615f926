/*
 * EngineJobCausalLog -- drop-in JobCausalLog (JobCausalLog.java:52-77) over the native engine,
 * with the semantics of JobCausalLogImpl (JobCausalLogImpl.java:71-266) and of its two delta
 * serde strategies (AbstractDeltaSerializerDeserializer.java:88-213, Flat :56-120, Grouping
 * :65-165).  JobCausalLogFactory (:56-67) swaps `new JobCausalLogImpl(...)` for
 * `new EngineJobCausalLog(engine, jobID, ...)`.
 *
 * What stays in Java: the flat and hierarchical maps of the job's thread logs (so the order
 * the strategies visit logs in -- ConcurrentHashMap iteration order -- is the reference's
 * own), the local-task table, the vertex distances and the pre-hasDelta filters of the
 * delta-sharing optimisations.  What moves to the engine:
 *   - every thread log's bytes and metadata (EngineThreadCausalLog);
 *   - enrichWithCausalLogDelta: the visit list of one outgoing buffer goes to clg_enrich_batch
 *     in one call (hasDelta + offset + slice of every log, header written by the engine);
 *   - processCausalLogDelta: one clg_process_delta call parses the header, applies every
 *     delta and opens the upstream logs not seen before; Java then registers the new logs in
 *     its maps exactly as insertNewUpstreamLog (:165-194) does;
 *   - notifyCheckpointComplete: the job's CAS and the fan-out to every log (clg_truncate_all).
 *
 * Source-only: this container has no JDK, so the binding is not compiled here.
 */
package org.apache.flink.runtime.causal.log.job;

import org.apache.flink.runtime.causal.DeterminantResponseEvent;
import org.apache.flink.runtime.causal.VertexGraphInformation;
import org.apache.flink.runtime.causal.VertexID;
import org.apache.flink.runtime.causal.determinant.DeterminantEncoder;
import org.apache.flink.runtime.causal.determinant.SimpleDeterminantEncoder;
import org.apache.flink.runtime.causal.engine.ClonosEngine;
import org.apache.flink.runtime.causal.log.job.hierarchy.PartitionCausalLogs;
import org.apache.flink.runtime.causal.log.job.hierarchy.VertexCausalLogs;
import org.apache.flink.runtime.causal.log.job.serde.DeltaEncodingStrategy;
import org.apache.flink.runtime.causal.log.thread.EngineThreadCausalLog;
import org.apache.flink.runtime.causal.log.thread.ThreadCausalLog;
import org.apache.flink.runtime.io.network.api.DeterminantRequestEvent;
import org.apache.flink.runtime.io.network.api.writer.ResultPartitionWriter;
import org.apache.flink.runtime.io.network.partition.consumer.InputChannelID;
import org.apache.flink.runtime.jobgraph.IntermediateResultPartitionID;
import org.apache.flink.runtime.jobgraph.JobVertexID;
import org.apache.flink.shaded.netty4.io.netty.buffer.ByteBuf;
import org.apache.flink.shaded.netty4.io.netty.buffer.ByteBufAllocator;
import org.apache.flink.shaded.netty4.io.netty.buffer.CompositeByteBuf;
import org.apache.flink.shaded.netty4.io.netty.buffer.Unpooled;

import java.nio.ByteBuffer;
import java.util.HashMap;
import java.util.Map;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.ConcurrentMap;
import java.util.stream.Collectors;

import static org.apache.flink.runtime.causal.engine.ClonosEngine.*;
import static org.apache.flink.runtime.causal.log.CausalLogManager.FULL_SHARING;

public class EngineJobCausalLog implements JobCausalLog {

	/** clg_enrich_batch / clg_process_delta strategies (include/clonos_engine.h). */
	private static final int CLG_DELTA_FLAT = 0;
	private static final int CLG_DELTA_HIERARCHICAL = 1;
	private static final byte CLG_DE_SEND = 1;

	private static final Object upstreamInsertLock = new Object(); // Abstract...:63

	private final ClonosEngine engine;
	private final int job;
	private final int determinantSharingDepth;
	private final DeterminantEncoder determinantEncoder;
	private final ByteBufAllocator alloc;
	private final int strategy;
	private final boolean enableDeltaSharingOptimizations;

	private final Map<Short, Integer> vertexIDToDistance = new HashMap<>();
	private final ConcurrentMap<CausalLogID, ThreadCausalLog> flatThreadCausalLogs = new ConcurrentHashMap<>();
	private final ConcurrentMap<Integer, EngineThreadCausalLog> byHandle = new ConcurrentHashMap<>();
	private final ConcurrentMap<Short, VertexCausalLogs> hierarchicalThreadCausalLogsToBeShared =
		new ConcurrentHashMap<>();
	private final ConcurrentMap<JobVertexID, Short> localTasks = new ConcurrentHashMap<>();
	private final Map<InputChannelID, CausalLogID> outputChannelSpecificCausalLogs = new ConcurrentHashMap<>();

	/** Grows to the largest delta seen; CLG_E_CAPACITY reports the size needed. */
	private static final int INITIAL_OUT = 4096;

	public EngineJobCausalLog(ClonosEngine engine, long jobIdLower, long jobIdUpper, int determinantSharingDepth,
							  DeltaEncodingStrategy deltaEncodingStrategy, boolean enableDeltaSharingOptimizations,
							  ByteBufAllocator alloc) {
		this.engine = engine;
		this.job = engine.openJob(jobIdLower, jobIdUpper, determinantSharingDepth);
		this.determinantSharingDepth = determinantSharingDepth;
		this.determinantEncoder = new SimpleDeterminantEncoder();
		this.alloc = alloc;
		this.strategy = deltaEncodingStrategy.equals(DeltaEncodingStrategy.FLAT) ? CLG_DELTA_FLAT
			: CLG_DELTA_HIERARCHICAL;
		this.enableDeltaSharingOptimizations = enableDeltaSharingOptimizations;
	}

	private EngineThreadCausalLog newLog(CausalLogID id) {
		EngineThreadCausalLog l = new EngineThreadCausalLog(engine, job, id, determinantEncoder, alloc);
		byHandle.put(l.handle(), l);
		return l;
	}

	/** JobCausalLogImpl.registerTask :124-169. */
	@Override
	public void registerTask(VertexGraphInformation vertexGraphInformation, JobVertexID jobVertexId,
							 ResultPartitionWriter[] resultPartitionsOfLocalVertex) {
		short vertexID = vertexGraphInformation.getThisTasksVertexID().getVertexID();
		localTasks.put(jobVertexId, vertexID);
		vertexIDToDistance.putAll(vertexGraphInformation.getDistances().entrySet().stream()
			.collect(Collectors.toMap(e -> e.getKey().getVertexID(), Map.Entry::getValue)));

		CausalLogID mainId = new CausalLogID(vertexID);
		ThreadCausalLog mainThreadLog = newLog(mainId);
		flatThreadCausalLogs.put(mainId, mainThreadLog);
		VertexCausalLogs v = null;
		if (determinantSharingDepth != 0) {
			v = new VertexCausalLogs(vertexID);
			hierarchicalThreadCausalLogsToBeShared.put(vertexID, v);
			v.mainThreadLog.set(mainThreadLog);
		}
		for (ResultPartitionWriter writer : resultPartitionsOfLocalVertex) {
			IntermediateResultPartitionID pid = writer.getPartitionId().getPartitionId();
			PartitionCausalLogs p = null;
			if (determinantSharingDepth != 0) {
				p = new PartitionCausalLogs(pid);
				v.partitionCausalLogs.put(pid, p);
			}
			for (int i = 0; i < writer.getNumberOfSubpartitions(); i++) {
				CausalLogID sid = new CausalLogID(vertexID, pid.getLowerPart(), pid.getUpperPart(), (byte) i);
				ThreadCausalLog s = newLog(sid);
				flatThreadCausalLogs.put(sid, s);
				if (determinantSharingDepth != 0)
					p.subpartitionLogs.put((byte) i, s);
			}
		}
	}

	@Override
	public ThreadCausalLog getThreadCausalLog(CausalLogID causalLogID) {
		return flatThreadCausalLogs.get(causalLogID);
	}

	/** AbstractDeltaSerializerDeserializer.processCausalLogDelta :118-139 in one engine call; the
	 *  logs it opened are registered as insertNewUpstreamLog (:165-194) does. */
	@Override
	public void processCausalLogDelta(ByteBuf msg) {
		if (determinantSharingDepth == 0)
			return;
		final int start = msg.readerIndex();
		final int headerBytes = msg.getInt(start);
		final int len = msg.readableBytes();
		final ByteBuf direct = msg.isDirect() && msg.nioBufferCount() == 1 ? msg
			: Unpooled.directBuffer(len).writeBytes(msg, start, len);
		final int[] handles = new int[headerBytes / 8 + 1]; // every log entry is more than 8 header bytes
		final long[] res = new long[3];
		try {
			ByteBuffer nio = direct.nioBuffer(direct == msg ? start : 0, len);
			check(nProcessDelta(engine.handle(), job, strategy, nio, 0, len, handles, res));
		} finally {
			if (direct != msg)
				direct.release();
		}
		msg.readerIndex(start + headerBytes); // where the reference's header walk stops (:135)
		final int n = (int) res[1];
		for (int i = 0; i < n; i++) {
			if (!byHandle.containsKey(handles[i])) {
				synchronized (upstreamInsertLock) {
					if (!byHandle.containsKey(handles[i]))
						insertNewUpstreamLog(handles[i]);
				}
			}
		}
	}

	private void insertNewUpstreamLog(int handle) {
		long[] w = new long[6];
		check(nLogGetId(engine.handle(), handle, w));
		final short vid = (short) w[0];
		final CausalLogID id = w[1] != 0 ? new CausalLogID(vid) : new CausalLogID(vid, w[2], w[3], (byte) w[4]);
		EngineThreadCausalLog l = EngineThreadCausalLog.wrap(engine, handle, id, determinantEncoder, alloc);
		byHandle.put(handle, l);
		flatThreadCausalLogs.put(id, l);
		int distance = Math.abs(vertexIDToDistance.get(vid));
		if (determinantSharingDepth == -1 || distance + 1 <= determinantSharingDepth) {
			VertexCausalLogs v = hierarchicalThreadCausalLogsToBeShared.computeIfAbsent(vid, VertexCausalLogs::new);
			if (id.isMainThread()) {
				v.mainThreadLog.set(l);
			} else {
				IntermediateResultPartitionID pid =
					new IntermediateResultPartitionID(id.getIntermediateDataSetLower(), id.getIntermediateDataSetUpper());
				v.partitionCausalLogs.computeIfAbsent(pid, PartitionCausalLogs::new).subpartitionLogs
					.putIfAbsent(id.getSubpartitionIndex(), l);
			}
		}
	}

	/** AbstractDeltaSerializerDeserializer.enrichWithCausalLogDelta :88-116: the strategy's visit
	 *  list is built here, the hasDelta / offset / slice of every log and the header are one
	 *  clg_enrich_batch call. */
	@Override
	public ByteBuf enrichWithCausalLogDelta(ByteBuf serialized, InputChannelID outputChannelID, long epochID,
											ByteBufAllocator alloc) {
		if (determinantSharingDepth == 0)
			return serialized;
		final CausalLogID channelLog = outputChannelSpecificCausalLogs.get(outputChannelID);
		final VisitList visit = new VisitList();
		if (strategy == CLG_DELTA_FLAT)
			visitFlat(channelLog, visit);
		else
			visitGrouping(channelLog, visit);

		final long[] req = {outputChannelID.getLowerPart(), outputChannelID.getUpperPart(), epochID, 0, visit.n};
		final long[] res = new long[4];
		final long[] total = new long[1];
		int cap = INITIAL_OUT;
		ByteBuf out = alloc.directBuffer(cap);
		int st = nEnrichBatch(engine.handle(), strategy, req, visit.logs(), visit.flags(), out.nioBuffer(0, cap), res,
			total);
		while (st == CLG_E_CAPACITY) { // nothing moved: fetch again at the size the engine needs
			out.release();
			cap = (int) total[0] + 256;
			out = alloc.directBuffer(cap);
			st = nEnrichBatch(engine.handle(), strategy, req, visit.logs(), visit.flags(), out.nioBuffer(0, cap), res,
				total);
		}
		if (st != CLG_OK || res[0] != CLG_OK) {
			out.release();
			check(st != CLG_OK ? st : (int) res[0]);
		}
		final int addedSize = (int) res[3]; // header + deltas
		out.writerIndex((int) res[2] + addedSize).readerIndex((int) res[2]);
		CompositeByteBuf composite = alloc.compositeDirectBuffer(Integer.MAX_VALUE);
		composite.addComponent(true, serialized);
		composite.addComponent(true, out);
		composite.setInt(0, composite.getInt(0) + addedSize);
		return composite;
	}

	/** FlatDeltaSerializerDeserializer.serializeDataStrategy :57-90 (pre-hasDelta filter). */
	private void visitFlat(CausalLogID channelLog, VisitList visit) {
		for (VertexCausalLogs v : hierarchicalThreadCausalLogsToBeShared.values()) {
			ThreadCausalLog main = v.mainThreadLog.get();
			if (main != null)
				visitFlatOne(channelLog, main, visit);
			for (PartitionCausalLogs p : v.partitionCausalLogs.values())
				for (ThreadCausalLog s : p.subpartitionLogs.values())
					visitFlatOne(channelLog, s, visit);
		}
	}

	private void visitFlatOne(CausalLogID channelLog, ThreadCausalLog log, VisitList visit) {
		CausalLogID cid = log.getCausalLogID();
		short vertex = cid.getVertexID();
		if (!enableDeltaSharingOptimizations || !localTasks.containsValue(vertex)
			|| (channelLog.isForVertex(vertex) && cid.isMainThread()) || channelLog.equals(cid))
			visit.add(((EngineThreadCausalLog) log).handle(), CLG_DE_SEND);
	}

	/** GroupingDeltaSerializerDeserializer.serializeDataStrategy :91-165: vertex-major, the main
	 *  log first, each partition's subpartitions contiguous; the post-hasDelta subpartition
	 *  filter (:148-151) becomes the entry's CLG_DE_SEND flag. */
	private void visitGrouping(CausalLogID channelLog, VisitList visit) {
		for (Map.Entry<Short, VertexCausalLogs> e : hierarchicalThreadCausalLogsToBeShared.entrySet()) {
			short vertexID = e.getKey();
			if (enableDeltaSharingOptimizations && localTasks.containsValue(vertexID)
				&& !channelLog.isForVertex(vertexID))
				continue;
			VertexCausalLogs v = e.getValue();
			ThreadCausalLog main = v.mainThreadLog.get();
			if (main != null)
				visit.add(((EngineThreadCausalLog) main).handle(), CLG_DE_SEND);
			for (PartitionCausalLogs p : v.partitionCausalLogs.values())
				for (ThreadCausalLog s : p.subpartitionLogs.values()) {
					boolean send = !enableDeltaSharingOptimizations || !channelLog.isForVertex(vertexID)
						|| channelLog.equals(s.getCausalLogID());
					visit.add(((EngineThreadCausalLog) s).handle(), send ? CLG_DE_SEND : 0);
				}
		}
	}

	/** JobCausalLogImpl.respondToDeterminantRequest :187-204. */
	@Override
	public DeterminantResponseEvent respondToDeterminantRequest(DeterminantRequestEvent e) {
		VertexID vertexId = e.getFailedVertex();
		long startEpochID = e.getStartEpochID();
		if (determinantSharingDepth != FULL_SHARING
			&& Math.abs(vertexIDToDistance.get(vertexId.getVertexID())) > determinantSharingDepth)
			return new DeterminantResponseEvent(e);
		short vertex = vertexId.getVertexID();
		Map<CausalLogID, ByteBuf> determinants = new HashMap<>();
		for (Map.Entry<CausalLogID, ThreadCausalLog> entry : flatThreadCausalLogs.entrySet())
			if (entry.getKey().isForVertex(vertex))
				determinants.put(entry.getKey(), entry.getValue().getDeterminants(startEpochID));
		return new DeterminantResponseEvent(e, determinants);
	}

	@Override
	public void registerDownstreamConsumer(InputChannelID outputChannelID, CausalLogID consumedLog) {
		outputChannelSpecificCausalLogs.put(outputChannelID, consumedLog);
	}

	@Override
	public void unregisterDownstreamConsumer(InputChannelID toCancel) {
		for (ThreadCausalLog l : flatThreadCausalLogs.values())
			l.unregisterConsumer(toCancel);
	}

	@Override
	public DeterminantEncoder getDeterminantEncoder() {
		return determinantEncoder;
	}

	@Override
	public int getDeterminantSharingDepth() {
		return determinantSharingDepth;
	}

	/** JobCausalLogImpl.notifyCheckpointComplete :229-246: the job's CAS and the fan-out run in
	 *  the engine (clg_truncate_all), so concurrent tasks of the job race exactly as on the
	 *  AtomicLong. */
	@Override
	public void notifyCheckpointComplete(long checkpointID) {
		engine.truncateAll(job, checkpointID);
	}

	@Override
	public int threadLogLength(CausalLogID causalLogID) {
		return flatThreadCausalLogs.get(causalLogID).logLength();
	}

	/** JobCausalLogImpl.unregisterTask :253-266. */
	@Override
	public synchronized boolean unregisterTask(JobVertexID jobVertexId) {
		boolean noMoreLocalTasks = false;
		if (localTasks.size() == 1) {
			for (ThreadCausalLog l : flatThreadCausalLogs.values())
				l.close();
			engine.closeJob(job);
			noMoreLocalTasks = true;
		}
		localTasks.remove(jobVertexId);
		return noMoreLocalTasks;
	}

	/** One outgoing buffer's visit list: engine log handles and CLG_DE_* flags. */
	private static final class VisitList {
		int[] logs = new int[64];
		byte[] flags = new byte[64];
		int n;

		void add(int log, byte flag) {
			if (n == logs.length) {
				logs = java.util.Arrays.copyOf(logs, 2 * n);
				flags = java.util.Arrays.copyOf(flags, 2 * n);
			}
			logs[n] = log;
			flags[n++] = flag;
		}

		int[] logs() {
			return n == logs.length ? logs : java.util.Arrays.copyOf(logs, n);
		}

		byte[] flags() {
			return n == flags.length ? flags : java.util.Arrays.copyOf(flags, n);
		}
	}
}
