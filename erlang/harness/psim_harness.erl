%% psim_harness -- the in-BEAM parity harness (SURVEY.md App. C): the
%% reference's own HyParView manager and Plumtree broadcast modules, driven
%% for N simulated nodes inside ONE BEAM process under the simulator's round
%% model R0 (DESIGN.md section 2), with the simulator's Philox stream as each
%% node's `rand` state.  It writes every emitted message of every round as a
%% record line in the engine's encoding, so erlang/harness/compare_trace.py
%% can diff it against the CPU oracle (and through it the GPU engine),
%% seed for seed.  It also exports erlang:phash(NodeSpec, 2^32) - 1 of every
%% node -- the sets v1 slots (16 buckets, or the linear hash's wider tables
%% past 80 elements) the engine's stand-in hash replaces.
%%
%% NOT RUN HERE: this image has no Erlang VM (SURVEY 8(c)).  Run recipe:
%% erlang/harness/README.md.
%%
%% The reference modules run unmodified; the harness replaces only what a
%% real deployment puts around them (shims/ is loaded ahead of the reference
%% ebin): partisan_config (per-node identity and config in the process
%% dictionary), partisan_peer_service_client (a connection = a recording
%% proxy), partisan_peer_service_events (notify -> the node's Plumtree state)
%% and, for Plumtree's send/3, the peer-service manager (psim_h_pt_manager).
%% HyParView callbacks are called as gen_server callbacks
%% (hv = src/partisan_hyparview_peer_service_manager.erl):
%%   init/1 (:289-354), handle_cast({join, Peer}) (:500-515),
%%   handle_cast({receive_message, M}) (:517-518),
%%   handle_info(random_promotion | passive_view_maintenance) (:542-607),
%%   handle_info({'EXIT', Pid, normal}) (:609-654)
%% and Plumtree's (pt = src/partisan_plumtree_broadcast.erl): init/1
%% (:251-264), handle_cast/2 (:282-336), handle_info(lazy_tick) (:341-345).
-module(psim_harness).
-export([main/1, run/2, spec/1, name/1, id_of/1, reachable/2, register_conn/3, record/3,
         pt_update/1, pt_send/4, have/1, have_add/1, write_buckets/2]).

-define(HV, partisan_hyparview_peer_service_manager).
-define(PT, partisan_plumtree_broadcast).
-define(NONE, 16#FFFFFFFF).
-define(MAP_BIT, 16#80000000).

%% HyParView's state record, field order of hv:88-101 (the harness reads
%% the active view and the connections of a node between callbacks)
-define(ST_ACTIVE, 3).
-define(ST_CONNECTIONS, 8).

%% erl -noshell -pa shims -pa <partisan ebin> -pa . -s psim_harness main Scenario Out
main([Scenario, Out]) ->
    {ok, Events} = file:consult(atom_to_list(Scenario)),
    ok = run(Events, atom_to_list(Out)),
    halt(0).

%% Events (file:consult terms):
%%   {config, #{n_nodes := N, seed := S, rounds := R, ...partisan_config keys}}
%%   {join, Round, [{Id, Contact | none}]}    start (init/1), then JOIN to Contact
%%   {crash, Round, [Id]}
%%   {partition, Round, [Group]}              one group per node, N entries
%%   {clear_partition, Round}
%%   {broadcast, Round, Root, MsgId}          plumtree_backend heartbeat at Root
run(Events, OutFile) ->
    [Cfg] = [C || {config, C} <- Events],
    #{n_nodes := N, seed := Seed, rounds := Rounds} = Cfg,
    process_flag(trap_exit, true),
    ets:new(partisan_connection_cache, [named_table, public, set]),   % partisan_connection_cache ETS
    put(psim_h_n, N),
    put(psim_h_seed, Seed),
    put(psim_h_part, maps:new()),
    [put({psim_h_cfg, K}, V) || {K, V} <- maps:to_list(maps:without([n_nodes, seed, rounds], Cfg))],
    put({psim_h_cfg, random_seed_int}, Seed),
    put({psim_h_cfg, broadcast_mods}, [psim_h_handler]),
    {ok, F} = file:open(OutFile, [write]),
    ok = write_buckets(F, N),
    Nodes = lists:foldl(fun(R, Acc) -> round(R, Events, Acc, F) end, #{}, lists:seq(0, Rounds - 1)),
    ok = write_views(F, Nodes),
    file:close(F).

%% ----------------------------------------------------------- one round
round(R, Events, Nodes0, F) ->
    put(psim_h_round, R),
    put(psim_h_out, []),
    put(psim_h_seq, #{}),
    Crashed = lists:append([Ids || {crash, RR, Ids} <- Events, RR =:= R]),
    %% events (R0 step 1): crashes, partition changes, starts, the origin
    Nodes1 = lists:foldl(fun(Id, Acc) -> crash(Id, Acc) end, Nodes0, Crashed),
    [put(psim_h_part, maps:from_list(lists:zip(lists:seq(0, get(psim_h_n) - 1), G)))
     || {partition, RR, G} <- Events, RR =:= R],
    [put(psim_h_part, maps:new()) || {clear_partition, RR} <- Events, RR =:= R],
    put(psim_h_nodes, Nodes1),
    Starts = lists:append([J || {join, RR, J} <- Events, RR =:= R]),
    Nodes2 = lists:foldl(fun({Id, C}, Acc) -> start(Id, C, R, Acc) end, Nodes1, Starts),
    Origin = [{Root, Msg} || {broadcast, RR, Root, Msg} <- Events, RR =:= R],
    Inbox = get(psim_h_inbox_next, #{}),
    put(psim_h_nodes, Nodes2),
    %% every running node in id order (R0 step 2)
    Nodes3 = lists:foldl(fun(Id, Acc) ->
                                 case maps:get(Id, Acc) of
                                     #{up := true} = Node ->
                                         put(psim_h_nodes, Acc),
                                         Acc#{Id => node_round(Id, Node, R, Crashed,
                                                               maps:get(Id, Inbox, []), Origin)};
                                     _ -> Acc
                                 end
                         end, Nodes2, lists:sort(maps:keys(Nodes2))),
    %% route (R0 step 3): this round's records, grouped by destination in
    %% (src, seq) order, are next round's inboxes
    Out = lists:reverse(get(psim_h_out)),
    [io:format(F, "R ~b ~b ~b ~b ~b ~b ~b ~b ~b ~b~s~n",
               [R, S, Q, D, T, TTL, A0, A1, A2, length(Ex), [[$\s | integer_to_list(X)] || X <- Ex]])
     || {S, Q, D, {T, TTL, A0, A1, A2, Ex}, _Msg} <- Out],
    put(psim_h_inbox_next,
        lists:foldl(fun({_S, _Q, D, _Rec, Msg}, Acc) ->
                            maps:update_with(D, fun(L) -> L ++ [Msg] end, [Msg], Acc)
                    end, #{}, Out)),
    Nodes3.

node_round(Id, Node0, R, Crashed, Msgs, Origin) ->
    #{hv := HV0, pt := PT0, ctr := Ctr0, start := Start, contact := Contact} = Node0,
    put(psim_h_node, Id),
    put(psim_h_pt, PT0),
    put(psim_h_have, maps:get(have, Node0)),
    psim_philox:install(get(psim_h_seed), Id, Ctr0),
    %% a. join (hv:500-515)
    HV1 = case Start =:= R andalso Contact =/= none of
              true -> noreply(?HV:handle_cast({join, spec(Contact)}, HV0));
              false -> HV0
          end,
    %% b. EXIT at every holder of a connection to a peer that crashed this
    %% round (App. A Q11): the active members holding one, in to_list order,
    %% then the node's other connections (lingering ones: a shuffle reply's
    %% Sender, a rejected requester, a pending promotion, the join contact),
    %% in id order -- their EXITs only edit the passive view and the
    %% connections, so their order among themselves does not matter; the
    %% oracle (psim_oracle.c process_node) runs them in the same sequence
    Active1 = [P || P <- sets:to_list(element(?ST_ACTIVE, HV1)), id_of(P) =/= Id],
    Others = lists:usort([D || {{S, D}, _} <- maps:to_list(get(psim_h_conn_map, #{})), S =:= Id,
                               not lists:member(D, [id_of(P) || P <- Active1])]),
    HV2 = lists:foldl(fun(P, H) ->
                              case lists:member(id_of(P), Crashed) of
                                  true ->
                                      case partisan_peer_service_connections:find(P, conns(H)) of
                                          {ok, [{_, _, Pid} | _]} ->
                                              noreply(?HV:handle_info({'EXIT', Pid, normal}, H));
                                          _ -> H
                                      end;
                                  false -> H
                              end
                      end, HV1, Active1 ++ [spec(D) || D <- Others]),
    %% connections to peers across the partition stay open but carry nothing
    %% this round (R0: the connect rule is evaluated when a message is sent):
    %% they are set aside for the node's round and put back after it
    {HV3, SetAside} = set_aside_unreachable(Id, HV2),
    Fresh = Start =:= R,                                      % a fresh incarnation drops its inbox
    {HvMsgs, PtMsgs} = lists:partition(fun is_hv/1, case Fresh of true -> []; false -> Msgs end),
    %% c. HyParView inbox
    HV4 = lists:foldl(fun(M, H) -> noreply(?HV:handle_cast({receive_message, M}, H)) end, HV3, HvMsgs),
    %% d, e. timers: random_promotion every 5 rounds, passive_view_maintenance every 10
    HV5 = case due(5, R, Start) of
              true -> noreply(?HV:handle_info(random_promotion, HV4));
              false -> HV4
          end,
    HV6 = case due(10, R, Start) of
              true -> noreply(?HV:handle_info(passive_view_maintenance, HV5));
              false -> HV5
          end,
    put(psim_h_hv, HV6),
    %% f. Plumtree inbox
    PT1 = lists:foldl(fun(M, P) -> noreply(?PT:handle_cast(M, P)) end, get(psim_h_pt), PtMsgs),
    %% g. origin: the backend's heartbeat (plumtree_backend:179-200) inserts
    %% the id, then broadcast/2 (pt:176-178)
    PT2 = case [Msg || {Root, Msg} <- Origin, Root =:= Id] of
              [Msg] ->
                  MsgId = {name(Id), Msg},
                  have_add(MsgId),
                  noreply(?PT:handle_cast({broadcast, MsgId, MsgId, psim_h_handler}, PT1));
              [] -> PT1
          end,
    %% h. lazy tick every round (pt:341-345)
    PT3 = case due(1, R, Start) of
              true -> noreply(?PT:handle_info(lazy_tick, PT2));
              false -> PT2
          end,
    {_, _, Ctr} = psim_philox:state(),
    Node0#{hv := put_back(SetAside, get(psim_h_hv)), pt := PT3, ctr := Ctr, have := get(psim_h_have)}.

noreply({noreply, S}) -> S.

due(Period, R, Start) -> R > Start andalso (R - Start) rem Period =:= 0.

is_hv(M) when is_tuple(M) ->
    lists:member(element(1, M), [join, forward_join, neighbor, disconnect, neighbor_request,
                                 neighbor_accepted, neighbor_rejected, shuffle, shuffle_reply]).

conns(HV) -> element(?ST_CONNECTIONS, HV).

set_aside_unreachable(Id, HV) ->
    {Conns, Aside} =
        lists:foldl(fun(P, {C, A}) ->
                            case {reachable(Id, P), partisan_peer_service_connections:find(name(P), C)} of
                                {false, {ok, Entries}} when Entries =/= [] ->
                                    {partisan_peer_service_connections:erase(name(P), C), [{P, Entries} | A]};
                                _ -> {C, A}
                            end
                    end, {conns(HV), []}, known_peers(Id)),
    {setelement(?ST_CONNECTIONS, HV, Conns), Aside}.

%% the set-aside connections back, unless the round made a new one to the
%% same peer (residual, unpinned: a disconnect/2 of a set-aside peer during
%% the round is not replayed on it)
put_back(Aside, HV) ->
    Conns = lists:foldl(fun({P, Entries}, C) ->
                                case partisan_peer_service_connections:find(name(P), C) of
                                    {ok, E} when E =/= [] -> C;
                                    _ -> lists:foldl(fun({A, Ch, Pid}, C1) ->
                                                             partisan_peer_service_connections:store(spec(P), {A, Ch, Pid}, C1)
                                                     end, C, Entries)
                                end
                        end, conns(HV), Aside),
    setelement(?ST_CONNECTIONS, HV, Conns).

known_peers(Id) -> [D || {{S, D}, _} <- maps:to_list(get(psim_h_conn_map, #{})), S =:= Id].

%% ------------------------------------------------------ node lifecycle
start(Id, Contact, R, Nodes) ->
    put(psim_h_node, Id),
    put(psim_h_have, #{}),
    %% init/1 seeds the stream (partisan_config:seed/0 -> draw 0) -- hv:289-354
    {ok, HV} = ?HV:init([]),
    {_, _, Ctr} = psim_philox:state(),
    Me = name(Id),
    {ok, PT} = ?PT:init([[Me], [Me], [], [psim_h_handler], [{lazy_tick_period, 1000},
                                                              {exchange_tick_period, 10000}]]),
    C = case Contact of none -> none; ?NONE -> none; _ -> Contact end,
    Nodes#{Id => #{hv => HV, pt => PT, ctr => Ctr, start => R, contact => C, up => true, have => #{}}}.

crash(Id, Nodes) ->
    case maps:get(Id, Nodes, undefined) of
        #{up := true} = N ->
            [begin unlink(P), exit(P, kill) end
             || {{_S, D}, P} <- maps:to_list(get(psim_h_conn_map, #{})), D =:= Id],
            Nodes#{Id := N#{up := false}};
        _ -> Nodes
    end.

%% ------------------------------------------------------ shim callbacks
spec(Id) ->
    #{name => name(Id),
      listen_addrs => [#{ip => ip(Id), port => 9090}],
      channels => [undefined], parallelism => 1}.

name(Id) -> list_to_atom(lists:flatten(io_lib:format("n~10..0B@sim", [Id]))).

%% 10.0.0.0 + Id: term order of the specs is id order below 2^27 (the
%% listen address decides it before the name), as psim_wire.cpp's ip_base + id
ip(Id) ->
    Ip = 16#0A000000 + Id,
    {Ip bsr 24, (Ip bsr 16) band 255, (Ip bsr 8) band 255, Ip band 255}.

id_of(#{name := Name}) -> id_of(Name);
id_of(Name) when is_atom(Name) ->
    [$n | Rest] = atom_to_list(Name),
    list_to_integer(lists:takewhile(fun(C) -> C >= $0 andalso C =< $9 end, Rest)).

reachable(Src, Dst) ->
    case maps:get(Dst, get(psim_h_nodes), undefined) of
        #{up := true} ->
            Part = get(psim_h_part),
            Src =/= Dst andalso maps:get(Src, Part, 0) =:= maps:get(Dst, Part, 0);
        _ -> false
    end.

register_conn(Src, Dst, Pid) ->
    put(psim_h_conn_map, maps:put({Src, Dst}, Pid, get(psim_h_conn_map, #{}))).

get(K, Default) ->
    case get(K) of
        undefined -> Default;
        V -> V
    end.

%% an emitted record of the running node: (src, seq) numbering as the engine's
record(Src, Dst, Msg) ->
    Seqs = get(psim_h_seq),
    Q = maps:get(Src, Seqs, 0),
    put(psim_h_seq, Seqs#{Src => Q + 1}),
    put(psim_h_out, [{Src, Q, Dst, enc(Msg), Msg} | get(psim_h_out)]),
    ok.

pt_update(Names) ->
    put(psim_h_pt, noreply(?PT:handle_cast({update, Names}, get(psim_h_pt)))).

%% Plumtree send/3 over the node's HyParView connections (forward_message,
%% hv:441-460 -> do_send_message/4 without maybe_connect): any connection of
%% the manager -- an active member's or a lingering one (App. A Q11) -- to a
%% running, reachable peer; a self-addressed atom finds no connection (Q6)
pt_send(Src, Name, _Kind, Msg) ->
    Dst = id_of(Name),
    HV = get(psim_h_hv),
    Conn = case partisan_peer_service_connections:find(name(Dst), conns(HV)) of
               {ok, [_ | _]} -> true;
               _ -> false
           end,
    case Conn andalso reachable(Src, Dst) of
        true -> record(Src, Dst, Msg);
        false -> {error, disconnected}
    end.

have(Id) -> maps:is_key(Id, get(psim_h_have)).
have_add(Id) -> put(psim_h_have, maps:put(Id, true, get(psim_h_have))).

%% ------------------------------------------------------ record encoding
%% The engine's record fields (include/partisan_gpu_sim.h message types,
%% oracle/psim_oracle.c hv_send / pt_send arguments): {Type, TTL, A0, A1, A2, Ex}
enc({join, _Me, _Tag, Epoch}) -> {0, 0, Epoch, 0, 0, []};
enc({forward_join, Peer, _Tag, Epoch, TTL, _Sender}) -> {1, TTL, id_of(Peer), Epoch, 0, []};
enc({neighbor, _Me, _Tag, Did, _Peer}) -> {2, 0, did(Did), 0, 0, []};
enc({disconnect, _Me, Did}) -> {3, 0, did(Did), 0, 0, []};
enc({neighbor_request, _Me, _Prio, _Tag, Did, Ex}) -> {4, 0, did(Did), 0, 0, ids(Ex)};
enc({neighbor_accepted, _Me, _Tag, Did, Ex}) -> {5, 0, did(Did), 0, 0, ids(Ex)};
enc({neighbor_rejected, _Me, Ex}) -> {6, 0, 0, 0, 0, ids(Ex)};
enc({shuffle, Ex, TTL, _Sender}) -> {7, TTL, 0, 0, 0, ids(Ex)};
enc({shuffle_reply, Ex, _Sender}) -> {8, 0, 0, 0, 0, ids(Ex)};
enc({broadcast, {_, Msg}, _M, _Mod, Round, Root, _From}) -> {9, 0, Msg, Round, ident(Root), []};
enc({prune, Root, _From}) -> {10, 0, 0, 0, ident(Root), []};
enc({i_have, {_, Msg}, _Mod, Round, Root, _From}) -> {11, 0, Msg, Round, ident(Root), []};
enc({ignored_i_have, {_, Msg}, _Mod, Round, Root, _From}) -> {12, 0, Msg, Round, ident(Root), []};
enc({graft, {_, Msg}, _Mod, Round, Root, _From}) -> {13, 0, Msg, Round, ident(Root), []}.

did({Epoch, Count}) -> (Epoch bsl 20) bor Count.
ids(Ex) -> [id_of(P) || P <- Ex].
ident(#{name := N}) -> id_of(N) bor ?MAP_BIT;     % a node_spec map (App. A Q6)
ident(N) when is_atom(N) -> id_of(N).

%% ------------------------------------------------------ exports
write_buckets(F, N) ->
    [io:format(F, "B ~b ~b~n", [Id, erlang:phash(spec(Id), 4294967296) - 1]) || Id <- lists:seq(0, N - 1)],
    ok.

write_views(F, Nodes) ->
    [begin
         HV = maps:get(hv, Node),
         io:format(F, "V ~b ~s | ~s~n",
                   [Id, string:join([integer_to_list(id_of(P)) || P <- sets:to_list(element(?ST_ACTIVE, HV))], " "),
                    string:join([integer_to_list(id_of(P)) || P <- sets:to_list(element(4, HV))], " ")])
     end || {Id, #{up := true} = Node} <- lists:sort(maps:to_list(Nodes))],
    ok.
